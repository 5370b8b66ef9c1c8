import sys, time; sys.path.insert(0, '.')
import torch
from sdf3d_amd import Renderer, abi, renderer as R, scenes
rd = Renderer("cuda:0")
f = scenes.config("C4", precision=abi.PRECISION_FAST)
res = {}
for n in (1, 8):
    t = R.tiling(1 % n, n, 8)
    bufs = [rd.render(f, t)[0] for _ in range(3)]
    streams = [torch.cuda.Stream() for _ in range(3)]
    for ns in (1, 2, 3):
        for rep in range(2):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            K = 100
            for i in range(K):
                b = i % ns
                rd.render(f, t, out=bufs[b], stream=streams[b])
            torch.cuda.synchronize()
            el = (time.perf_counter() - t0) / K * 1e3
        res[f"share 1/{n}, {ns} streams"] = round(el, 4)
for k, v in res.items(): print(k, "ms/frame", v)
