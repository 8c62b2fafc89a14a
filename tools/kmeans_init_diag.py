"""KMeans init/convergence diagnostics on the bench data: coverage of the true mixture centres by the
k-means|| init, then per-step max centroid shift for the HIP path and the torch reference path."""
import argparse, json, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from alink_amd import useLocalEnv, RandomVectorSourceBatchOp
from alink_amd.models.clustering import kmeans as km
from alink_amd.ops import kmeans as kops

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=100_000_000)
ap.add_argument("--k", type=int, default=100)
ap.add_argument("--iters", type=int, default=20)
ap.add_argument("--init-steps", type=int, default=5)
ap.add_argument("--torch", action="store_true")
a = ap.parse_args()
env = useLocalEnv(1)
src = RandomVectorSourceBatchOp().setNumRows(a.rows).setSize(128).setNumClusters(a.k) \
    .setClusterStd(1.0).setCenterScale(4.0).setDtype("bf16").setSeed(2024).setOutputCol("vec")
X = src.getOutputTable().col("vec").values
g = torch.Generator(device="cpu").manual_seed(2024)
true_c = (torch.randn(a.k, 128, generator=g, dtype=torch.float64) * 4.0).to(X.device)
cand_info = {}
_orig = km._local_kmeans
def _spy(samples, w, k, dt, **kw):
    dd = torch.cdist(true_c, samples.to(true_c.dtype))
    cand_info.update(n_cand=int(samples.shape[0]), cand_covered=len(set(dd.argmin(1).tolist())))
    return _orig(samples, w, k, dt, **kw)
km._local_kmeans = _spy
t = time.perf_counter()
C = km.kmeans_init(X, a.k, "K_MEANS_PARALLEL", a.init_steps, "EUCLIDEAN")
t_init = time.perf_counter() - t
d = torch.cdist(true_c, C)
res = {"init_s": t_init, "init_k": C.shape[0], "covered": len(set(d.argmin(1).tolist())),
       "max_true_to_init": float(d.min(1).values.max()), **cand_info}
for path in (["hip", "torch"] if a.torch else ["hip"]):
    Cc = C.clone()
    shifts = []
    for it in range(a.iters):
        buf = kops.assign_accumulate(X, Cc) if path == "hip" else kops.assign_accumulate_torch(X, Cc)
        cnt = buf[:, -1]
        keep = cnt > 0
        Cn = buf[keep, :-1] / cnt[keep, None]
        sh = float((Cn - Cc[keep]).norm(dim=1).max()) if Cn.shape == Cc.shape else float("nan")
        shifts.append(sh)
        Cc = Cn
        if sh < 1e-4:
            break
    res[path] = {"iters": len(shifts), "shifts": shifts[:6] + shifts[-4:]}
print(json.dumps(res), flush=True)
