"""CPU model (analysis only, no GPU): where config 5's cancels point. Replays the config-5 stream for the
first N symbols through a price-time book (sortedcontainers) in 20-batch groups and classifies every cancel:
its target rested in the same group or an earlier one, and whether its level was taken from (in this group)
between the target's rest (or the group start) and the cancel — the cases a grouped walk that handles cancels
must resolve from FIFO positions.   python tools/c5_cancel_model.py [N]
"""
import os
import numpy as np, sys, collections
from sortedcontainers import SortedDict
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import matching_engine_amd as me
NS = int(sys.argv[1]) if len(sys.argv) > 1 else 256
sc = me.preset(5)
st = me.Stream(sc)
base = st.base_prices()
S = sc.num_symbols
bids = [SortedDict() for _ in range(S)]  # price -> deque[[seq, qty]]
asks = [SortedDict() for _ in range(S)]
where = {}  # seq -> (sym, side, price)
G = 20
stats = collections.Counter()
grp_bad_frac = []
for grp in range(4):
    bad = np.zeros(S, bool)
    last_take = [dict() for _ in range(S)]
    restt = {}
    t = 0
    for bi in range(G):
        B = st.next(sc.batch)
        sel = B.symbol < NS
        for i in np.nonzero(sel)[0]:
            s = int(B.symbol[i]); k = int(B.kind[i]); q = int(B.qty[i]); px = int(B.price_q4[i]); seq = int(B.seq[i])
            t += 1
            if (k >> 3) & 1:
                w = where.get(px)
                if w is None or w[0] != s:
                    stats['cx_unknown'] += 1; continue
                _, side, p = w
                lt = last_take[s].get((side, p))
                if px in restt:
                    ok = lt is None or lt < restt[px]
                    stats['cx_in_ok' if ok else 'cx_in_touched'] += 1
                else:
                    ok = lt is None
                    stats['cx_pre_ok' if ok else 'cx_pre_touched'] += 1
                if not ok and grp > 0: bad[s] = True
                book = bids[s] if side == 1 else asks[s]
                dq = book[p]
                for e in dq:
                    if e[0] == px: dq.remove(e); break
                if not dq: del book[p]
                del where[px]
                continue
            buy = (k & 3) == 1; mkt = (k >> 2) & 1
            rem = q
            opp = asks[s] if buy else bids[s]
            while rem and opp:
                p = opp.peekitem(0)[0] if buy else opp.peekitem(-1)[0]
                if not mkt and ((buy and p > px) or ((not buy) and p < px)): break
                dq = opp[p]
                last_take[s][(2 if buy else 1, p)] = t
                while rem and dq:
                    e = dq[0]
                    f = min(rem, e[1]); rem -= f; e[1] -= f
                    if e[1] == 0:
                        dq.popleft(); where.pop(e[0], None)
                if not dq: del opp[p]
            if rem and not mkt:
                own = bids[s] if buy else asks[s]
                if px not in own: own[px] = collections.deque()
                own[px].append([seq, rem])
                where[seq] = (s, 1 if buy else 2, px)
                restt[seq] = t
    if grp > 0: grp_bad_frac.append(bad[:NS].mean())
tot = sum(v for k, v in stats.items() if k.startswith('cx'))
for k, v in sorted(stats.items()): print(k, v, f"{100*v/tot:.1f}%")
print("symbol-groups with a touched-level cancel:", grp_bad_frac)
