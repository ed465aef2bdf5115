"""CPU model (analysis only, no GPU): config 4's hot symbol (seeded to 10,000 levels per side) — record paths,
and the distance from each emptied level to the next occupied one (what the ladder's next-level scan crosses)
and the spread.   python tools/c4_gap_model.py
"""
import os
import numpy as np, sys, collections
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import matching_engine_amd as me
sc = me.preset(4)
st = me.Stream(sc)
base = st.base_prices()
L = sc.levels
sb = st.seed_books([0], 10000)
t = np.zeros(L, dtype=np.int64)
b0 = int(base[0])
for i in range(len(sb)):
    off = int(sb.price_q4[i]) - b0
    t[off] += int(sb.qty[i])
occ = np.nonzero(t)[0]
print("seeded levels", len(occ), "range", occ.min(), occ.max())
def best():
    # bids below asks: find the split: asks are levels above max bid... we track sides separately
    pass
# determine sides: seed kinds
sides = {}
for i in range(len(sb)):
    off = int(sb.price_q4[i]) - b0
    sides[off] = int(sb.kind[i]) & 3
bidlv = sorted(l for l, s in sides.items() if s == 1)
asklv = sorted(l for l, s in sides.items() if s == 2)
print("bid range", bidlv[0], bidlv[-1], "ask range", asklv[0], asklv[-1])
bb = bidlv[-1]; ba = asklv[0]
gaps=[]; spreads=[]; C = collections.Counter(); pops = 0; nrec = 0; listdepth = collections.Counter()
for bi in range(6):
    B = st.next(sc.batch)
    sel = np.nonzero(B.symbol == 0)[0]
    for i in sel:
        k = int(B.kind[i]); q = int(B.qty[i]); px = int(B.price_q4[i])
        if (k >> 3) & 1: C['cancel'] += 1; continue
        buy = (k & 3) == 1; mkt = (k >> 2) & 1
        off = px - b0
        if not mkt and not (0 <= off < L): C['outside'] += 1; continue
        lim = (L - 1 if buy else 0) if mkt else off
        rem = q; e = 0
        if buy:
            while rem and ba < L and ba <= lim:
                if t[ba] > rem: t[ba] -= rem; rem = 0
                else:
                    rem -= t[ba]; t[ba] = 0; e += 1
                    nx = np.nonzero(t[ba+1:])[0]; gaps.append(nx[0]+1 if len(nx) else -1); ba = ba + 1 + nx[0] if len(nx) else L
        else:
            while rem and bb >= 0 and bb >= lim:
                if t[bb] > rem: t[bb] -= rem; rem = 0
                else:
                    rem -= t[bb]; t[bb] = 0; e += 1
                    nx = np.nonzero(t[:bb])[0]; gaps.append(bb-nx[-1] if len(nx) else -1); bb = nx[-1] if len(nx) else -1
        pops += e; nrec += 1; spreads.append(ba-bb)
        r = 'none'
        if rem and not mkt:
            if buy:
                if lim > bb: r = 'newbest'; bb = lim
                else:
                    d = np.count_nonzero(t[lim:bb+1]); r = 'atbest' if lim == bb else ('list' if d < 64 else 'deep')
            else:
                if lim < ba: r = 'newbest'; ba = lim
                else:
                    d = np.count_nonzero(t[ba:lim+1]); r = 'atbest' if lim == ba else ('list' if d < 64 else 'deep')
            t[lim] += rem
        C[('mkt' if mkt else 'lim', 'take%d' % min(e, 3) if e or rem < q else 'notake', r)] += 1
print("records", nrec, "pops/record", pops / nrec)
for k, v in sorted(C.items(), key=lambda x: -x[1])[:20]: print(k, v, f"{100*v/nrec:.1f}%")

g=np.array(gaps); print("pops", len(g), "gap mean", g.mean(), "p50", np.percentile(g,50), "p90", np.percentile(g,90), "p99", np.percentile(g,99), "scan iters mean", np.mean((g+63)//64))
sp=np.array(spreads); print("spread mean", sp.mean(), "p50", np.percentile(sp,50), "p90", np.percentile(sp,90))
