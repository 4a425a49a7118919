import sys, numpy as np
sys.path.insert(0, '.')
import __graft_entry__ as ge
g = ge.load_package()
from oracle import oracle_py as O
s = g.Scene("cornell", width=64)
cam = s.camera
ctx = g.Context(0); ctx.upload(s.desc)
h = s.hittables()
tg, pg, t_g = ctx.primary_hits(cam, 1234, 0)
to, po, t_o = O.primary_hits(s.desc, cam, 1234, 0, fp32=True)
mism = np.flatnonzero((tg != to) | (pg != po))
print("n mism", mism.size)
for i in mism[:12]:
    print(i, "gpu", tg[i], pg[i], h['kind'][pg[i]] if pg[i]>=0 else -1, t_g[i], "| ora", to[i], po[i], h['kind'][po[i]] if po[i]>=0 else -1, t_o[i])
# also compare with the old (mega) path? probe kernel uses same traverse
