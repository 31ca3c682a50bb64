import os, sys, numpy as np
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "tests"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "bipartite-link-prediction_amd"))
sys.path.insert(0, os.path.join(os.environ.get("GRAFT_REPO_ROOT", "/root/repo"), "oracle"))
import blp, blp_oracle as bo
from helpers import bipartite_edges
rng = np.random.default_rng(3)
a, b = bipartite_edges(rng, 3000, 300, 20000)
G = blp.DeviceGraph(a, b)
adj = {}
for x, y in zip(a.tolist(), b.tolist()):
    adj.setdefault(x, set()).add(y); adj.setdefault(y, set()).add(x)
src = G.n_col0 + np.arange(G.n - G.n_col0)
exp = [bo.topk_full_candidates(adj, int(G.node_ids[x]), 10, "common_neighbors")[1] for x in src]
for knobs in [{}, {"BLP_TOPK_DENSE_MAX": "1"}, {"BLP_TOPK_DENSE_MAX": "2"}, {"BLP_TOPK_NO_FUSE": "1"}, {"BLP_TOPK_NO_DENSE": "1"}, {"BLP_TOPK_EXPAND": "0"}]:
    for k in ("BLP_TOPK_DENSE_MAX", "BLP_TOPK_NO_FUSE", "BLP_TOPK_NO_DENSE", "BLP_TOPK_EXPAND"):
        os.environ.pop(k, None)
    os.environ.update(knobs)
    T = blp.TopK(G, "business")
    for mask in (blp.CN, blp.CN | blp.JACCARD | blp.ADAMIC):
        res = T(src, k=10, mask=mask)
        nc = res["common_neighbors"][2]
        bad = [(int(src[i]), int(nc[i]), exp[i]) for i in range(len(src)) if nc[i] != exp[i]]
        print(knobs, mask, "bad", len(bad), bad[:4], "dense adds", T.stats(7)[1], flush=True)
    T.close()
