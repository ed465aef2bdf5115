"""CPU model (analysis only, no GPU): the ladder walk's record paths on config 2's stream — partial takes,
levels emptied, rests at / above / below the best — per record.   python tools/c2_path_model.py
"""
import os
import numpy as np, sys, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import matching_engine_amd as me
sc = me.preset(2)
st = me.Stream(sc)
base = st.base_prices()
L = sc.levels
S = sc.num_symbols
# per symbol ladder of totals; bids below asks
tot = np.zeros((S, L), dtype=np.int64)
bb = np.full(S, -1); ba = np.full(S, L)
C = collections.Counter()
nb = 30
for b in range(nb):
    B = st.next(sc.batch)
    for i in range(len(B)):
        s = int(B.symbol[i]); k = int(B.kind[i]); q = int(B.qty[i]); px = int(B.price_q4[i])
        side = k & 3; mkt = (k >> 2) & 1; cancel = (k >> 3) & 1
        if cancel: C['cancel'] += 1; continue
        buy = side == 1
        off = px - int(base[s])
        lim = (L - 1 if buy else 0) if mkt else off
        if not mkt and not (0 <= off < L): C['outside'] += 1; continue
        tag = ('B' if buy else 'S') + ('M' if mkt else 'L')
        rem = q; emptied = 0; took = False
        t = tot[s]
        if buy:
            while rem and ba[s] < L and ba[s] <= lim:
                took = True
                l = ba[s]
                if t[l] > rem: t[l] -= rem; rem = 0
                else:
                    rem -= t[l]; t[l] = 0; emptied += 1
                    nx = np.nonzero(t[l+1:])[0]; ba[s] = l + 1 + nx[0] if len(nx) else L
                    if ba[s] < L and ba[s] <= bb[s]: pass
        else:
            while rem and bb[s] >= 0 and bb[s] >= lim:
                took = True
                l = bb[s]
                if t[l] > rem: t[l] -= rem; rem = 0
                else:
                    rem -= t[l]; t[l] = 0; emptied += 1
                    nx = np.nonzero(t[:l])[0]; bb[s] = nx[-1] if len(nx) else -1
        take = 'none' if not took else ('partial' if emptied == 0 else f'empty{min(emptied,3)}')
        rest = 'none'
        if rem and not mkt:
            if buy:
                rest = 'atbest' if lim == bb[s] else ('newbest' if lim > bb[s] else 'deep')
                if lim > bb[s]: bb[s] = lim
            else:
                rest = 'atbest' if lim == ba[s] else ('newbest' if lim < ba[s] else 'deep')
                if lim < ba[s]: ba[s] = lim
            t[lim] += rem
        if b >= 5: C[(take, rest)] += 1
tot_n = sum(v for k, v in C.items() if isinstance(k, tuple))
for k, v in sorted(C.items(), key=lambda x: -x[1]): print(k, v, f"{100*v/max(tot_n,1):.1f}%")
