"""Where do prefix-cached and per-row-prefilled rollouts part? (tests/test_prefix_cache_gpu.py, sampled bf16)

1. prefill of the 5 distinct prompts vs of all 40 rows: last hidden state and every layer's prompt keys / values;
2. rollouts with prefix caching on / off under each decode form (eager unpacked, graphed unpacked, graphed packed):
   first differing response position per form."""

import sys

import torch

sys.path.insert(0, ".")
from dots.rl_amd.config import to_attr  # noqa: E402
from dots.rl_amd.protocol import DataProto  # noqa: E402
from dots.rl_amd.qwen2 import KVCache, KVCacheRows, ParamStore, Qwen2Config, Qwen2Model  # noqa: E402
from dots.rl_amd.rollout import MI355XRollout  # noqa: E402

DEV = "cuda"
BF = torch.bfloat16
cfg = Qwen2Config.from_dict(dict(vocab_size=512, hidden_size=128, intermediate_size=256, num_hidden_layers=2,
                                 num_attention_heads=2, num_key_value_heads=1, max_position_embeddings=512,
                                 rope_theta=10000.0, rms_norm_eps=1e-6, tie_word_embeddings=True))
store = ParamStore(cfg, DEV, compute_dtype=BF, trainable=False)
store.init_random(4)
m = Qwen2Model(cfg, store)
n, nprompt, R = 8, 5, 20
for P in (40, 64):
    g = torch.Generator(device=DEV).manual_seed(P)
    ids = torch.randint(3, 512, (nprompt, P), device=DEV, generator=g)
    am = torch.ones(nprompt, P, dtype=torch.int64, device=DEV)
    for p in range(nprompt):
        am[p, : 3 * p] = 0
        ids[p, : 3 * p] = 0
    pos = (am.cumsum(-1) - 1).clamp_min(0)
    rep = lambda t: t.repeat_interleave(n, 0)  # noqa: E731
    B = n * nprompt
    ca = KVCache(cfg, B, P + R, DEV, BF)
    ha = m.prefill(ca, rep(ids), rep(am), rep(pos))
    cb = KVCache(cfg, B, P + R, DEV, BF)
    hb = m.prefill(KVCacheRows(cb, 0, nprompt), ids, am, pos)
    src = torch.arange(B, device=DEV) // n
    print(f"P={P}: h equal {torch.equal(ha, hb[src])}, max|dh| {(ha.float() - hb[src].float()).abs().max().item():.3g}")
    for i in range(cfg.num_hidden_layers):
        ka, kb = ca.k[i][:, :, :P], cb.k[i][src][:, :, :P]
        va = ca.vt[i][:, :, : (P + 31) // 32]
        vb = cb.vt[i][src][:, :, : (P + 31) // 32]
        print(f"  layer {i}: k equal {torch.equal(ka, kb)} vt equal {torch.equal(va, vb)}")
    for form in (dict(use_hip_graph=False, packed_decode=False), dict(use_hip_graph=True, packed_decode=False),
                 dict(use_hip_graph=True, packed_decode=True)):
        outs = []
        for share in (True, False):
            rcfg = to_attr(dict(do_sample=True, temperature=1.0, top_k=-1, top_p=1.0, response_length=R, n=n,
                                ignore_eos=False, seed=11, val_kwargs={}, enable_prefix_caching=share, **form))
            ro = MI355XRollout(m, rcfg)
            out = ro.generate_sequences(DataProto.from_dict(
                {"input_ids": rep(ids), "attention_mask": rep(am), "position_ids": rep(pos)},
                meta_info={"eos_token_id": 2, "pad_token_id": 0}))
            outs.append(out.batch["responses"])
        d = (outs[0] != outs[1])
        cols = d.any(0).nonzero().flatten().tolist()
        rows = d.any(1).nonzero().flatten().tolist()
        print(f"  {form}: differing rows {rows} first column {cols[:1]}")
