"""Which parameters differ between two identical trainer steps (concurrent weight gradients on): per named
parameter, the count of differing master entries, plus the first mini-batch's gradient (captured before the
optimizer step through FlatAdamW.step)."""
import sys

import torch

sys.path.insert(0, ".")
sys.path.insert(0, "tests")
from test_estimators_gpu import _trainer  # noqa: E402

runs = []
for r in range(3):
    tr = _trainer("grpo", ["actor_rollout_ref.actor.use_kl_loss=True"])
    w = tr.actor_rollout_wg.worker
    opt = w.actor_optimizer
    grads = []
    orig = opt.step

    def step(*a, _orig=orig, **k):
        torch.cuda.synchronize()
        grads.append(w.store.grad.clone())
        return _orig(*a, **k)

    opt.step = step
    tr.fit(num_steps=1)
    runs.append((w.store.master.clone(), grads, w.store))
m0, g0, store = runs[0]
for r in range(1, len(runs)):
    m1, g1, _ = runs[r]
    print(f"run {r}: grads per optimizer step equal:", [torch.equal(a, b) for a, b in zip(g0, g1)],
          "max rel grad diff:", [((a - b).abs().max() / a.abs().max()).item() for a, b in zip(g0, g1)])
    for name, (o, shape, kind) in store.offsets.items():
        n = 1
        for d in shape:
            n *= d
        for gi, (a, b) in enumerate(zip(g0, g1)):
            dd = (a[o:o + n] != b[o:o + n]).sum().item()
            if dd:
                print(f"   step {gi} grad {name} {kind}: {dd} of {n} differ, max {(a[o:o+n]-b[o:o+n]).abs().max().item():.3e}"
                      f" of {a[o:o+n].abs().max().item():.3e}")
