import sys, os, torch, torch.nn.functional as F
sys.path.insert(0, os.getcwd())
sys.path.insert(0, os.path.join(os.getcwd(), "tools"))
from kernel_bench import time_graph
import torch.cuda.tunable as tunable
from dots.rl_amd.workers import _enable_gemm_tuning
dev, bf = "cuda", torch.bfloat16
emb = torch.randn(151936, 896, device=dev, dtype=bf)
h = torch.randn(64, 896, device=dev, dtype=bf)
def t_eager(fn, n=20):
    fn(); torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(n): fn()
    b.record(); b.synchronize(); return a.elapsed_time(b) / n * 1e3
print("no tuning eager", t_eager(lambda: F.linear(h, emb)), "graph", time_graph(lambda: F.linear(h, emb), 20) * 1e6)
_enable_gemm_tuning("auto")
print("enabled", tunable.is_enabled(), tunable.tuning_is_enabled(), len(tunable.get_results()))
print("tuned eager", t_eager(lambda: F.linear(h, emb)), "graph", time_graph(lambda: F.linear(h, emb), 20) * 1e6)
h3 = torch.randn(64, 1, 896, device=dev, dtype=bf)[:, 0]
print("view eager", t_eager(lambda: F.linear(h3, emb)))
print([r for r in tunable.get_results() if "151936_64" in r[1]])
