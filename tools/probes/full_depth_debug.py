"""Debug: where does the fp32 full-depth model leave the reference (teacher-forced vs rollout)."""
import os, sys, json
import numpy as np, torch
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT); sys.path.insert(0, os.path.join(ROOT, "tests")); sys.path.insert(0, os.path.join(ROOT, "tests", "golden"))
import test_full_depth_gpu as t
z = np.load(os.path.join(ROOT, "tests/golden/full_depth.npz")); meta = json.loads(str(z["__meta__"]))
import full_depth as fd
sd = fd.make_state_dict()
for dt in (torch.float32,):
    m = t._model(sd, dt)
    lp, ent, am = t._teacher_forced(m, z)
    print("teacher-forced logp max diff", np.abs(lp - z["log_probs"]).max(), "argmax==ref", (am == z["responses"]).mean())
    print("per-row first argmax mismatch", [int(np.nonzero(am[b] != z["responses"][b])[0][0]) if (am[b] != z["responses"][b]).any() else -1 for b in range(4)])
    out, ro = t._rollout(m, z, meta)
    r = out.batch["responses"].cpu().numpy()
    print("rollout first mismatch", [int(np.nonzero(r[b] != z["responses"][b])[0][0]) if (r[b] != z["responses"][b]).any() else -1 for b in range(4)])
    print(r[:, :6]); print(z["responses"][:, :6])
    out, ro = t._rollout(m, z, meta, use_hip_graph=False)
    r = out.batch["responses"].cpu().numpy()
    print("eager rollout first mismatch", [int(np.nonzero(r[b] != z["responses"][b])[0][0]) if (r[b] != z["responses"][b]).any() else -1 for b in range(4)])
