"""Member skew and hand-off latency of the team exchange from TEAM_STAMP=3 dumps (BCMPC_STAMP_DUMP).
usage: python tools/team_xchg_stamps.py <dump file> <members T>
Each record: int32 [blocks, waves, H, K] + uint64 [blocks][waves][10] s_memrealtime values (100 MHz) of wave 0
(slots 5 d + k, steps H/2 + d: 0 partials done, 1 published, 2 own members in, 3 every member in, 4 totals)."""
import sys
import numpy as np

path, T = sys.argv[1], int(sys.argv[2])
raw = open(path, "rb").read()
off, recs = 0, []
while off < len(raw):
    b, w, H, K = np.frombuffer(raw, np.int32, 4, off)
    off += 16
    a = np.frombuffer(raw, np.uint64, b * w * 10, off).reshape(b, w, 10).astype(np.int64)
    off += b * w * 10 * 8
    recs.append(a)
a = recs[-1]                                   # the last stamped launch
blocks = a.shape[0]
rows = []
for d in (0, 1):
    s = a[:, 0, 5 * d:5 * d + 5]               # wave 0 of every block
    ok = (s > 0).all(axis=1)
    for c0 in range(blocks):
        pass
    # column c's members: blocks b with ((b >> 3) // T) * 8 + (b & 7) == c
    cols = {}
    for bb in range(blocks):
        if not ok[bb]:
            continue
        c = ((bb >> 3) // T) * 8 + (bb & 7)
        cols.setdefault(c, []).append(s[bb])
    for c, ms in cols.items():
        if len(ms) != T:
            continue
        m = np.array(ms) * 10.0 / 1000.0       # -> us
        pub = m[:, 1]
        rows.append(dict(
            skew_partials=m[:, 0].max() - m[:, 0].min(),
            skew_publish=pub.max() - pub.min(),
            sum_publish=(m[:, 1] - m[:, 0]).mean(),
            last_pub_to_all_in=(m[:, 3] - pub.max()).mean(),
            own_to_all_in=(m[:, 3] - m[:, 1]).mean(),
            wave0_poll=(m[:, 2] - m[:, 1]).mean(),
            after=(m[:, 4] - m[:, 3]).mean(),
            step=(m[:, 0].mean())))
keys = ["skew_partials", "skew_publish", "sum_publish", "wave0_poll", "own_to_all_in", "last_pub_to_all_in", "after"]
print(f"{len(rows)} column-steps (T = {T}); us, median [p10, p90]:")
for k in keys:
    v = np.array([r[k] for r in rows])
    print(f"  {k:20s} {np.median(v):6.2f} [{np.percentile(v, 10):6.2f}, {np.percentile(v, 90):6.2f}]")
