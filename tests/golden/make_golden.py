"""Generate golden vectors by running the REFERENCE implementation (dots.rl / verl) on seeded inputs.

Run in the survey/build container only (it needs ``/root/reference``; the GPU box never runs it):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

Every fixture stores its inputs and the reference's outputs as plain arrays (``.npz``, no pickles).
Reference call sites (file:line under /root/reference):

* policy loss / agg / KL / total actor loss + backward : verl/trainer/ppo/core_algos.py:703-736, 815-889, 1272-1307
  composed exactly as verl/workers/actor/dp_actor.py:419-466 does.
* GRPO advantage : verl/trainer/ppo/core_algos.py:260-324
* GAE + masked_whiten : verl/trainer/ppo/core_algos.py:208-256, verl/utils/torch_functional.py:171-223
* log-prob / entropy over vocab (+ backward) : verl/utils/torch_functional.py:116-160
* fused lm_head -> logp/entropy (+ backward) : verl/utils/experimental/torch_functional.py:20-216
* response mask / position ids : verl/utils/torch_functional.py:226-246, verl/utils/model.py:219,
  verl/workers/rollout/hf_rollout.py:151-160
* critic value loss + backward : verl/trainer/ppo/core_algos.py:1230-1269 as dp_critic.py:218-245 scales it
* critic forward/backward (tiny Qwen2ForTokenClassification, the model fsdp_workers.py:1003-1060 builds) :
  verl/workers/critic/dp_critic.py:57-145 values slice, compute_value_loss, loss.backward()
* DAPO overlong-buffer reward : verl/workers/reward_manager/dapo.py:60-150 (stub tokenizer / preset scores)
* Karmarkar-Karp balancing : verl/utils/seqlen_balancing.py:26-239 (partitions + imbalance metrics)
* RLOO / REINFORCE++-baseline advantages : verl/trainer/ppo/core_algos.py:392-493
* OPO / GPG / GRPO pass@k / ReMax advantages : verl/trainer/ppo/core_algos.py:327-386, 495-546, 588-684
* GSPO / GMPO (geo_mean) policy losses : verl/trainer/ppo/core_algos.py:892-954, 1143-1210
* Clip-Cov / KL-Cov policy losses : verl/trainer/ppo/core_algos.py:978-1140
* masked_mean known answers : tests/utils/test_torch_functional.py:55-66 (reference test, reproduced as data)
* rollout-vs-actor debug metrics : verl/utils/debug/metrics.py:63-108
* bf16 production-path update (fp32 and autocast-bf16 reference runs) : verl/workers/actor/dp_actor.py:110, 300-482
* configs #4 / #5 at full depth (Llama-3-8B, Qwen2.5-7B; fp32 and CPU-bf16 teacher-forced log-probs) : HF models as
  fsdp_workers.py:244-330 loads them
"""

import hashlib
import json
import os
import sys

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import _ref_stubs  # noqa: E402

DictConfig = _ref_stubs.install()

import verl.trainer.ppo.core_algos as ca  # noqa: E402
import verl.utils.experimental.torch_functional as vxf  # noqa: E402
import verl.utils.torch_functional as vF  # noqa: E402
from verl.utils.model import compute_position_id_with_mask  # noqa: E402

torch.set_num_threads(8)


def _save(name, arrays, meta):
    arrays = {k: (v.detach().cpu().numpy() if torch.is_tensor(v) else np.asarray(v)) for k, v in arrays.items()}
    arrays["__meta__"] = np.array(json.dumps(meta))
    path = os.path.join(HERE, name)
    np.savez_compressed(path, **arrays)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


# --------------------------------------------------------------------------------------------
# A10-A13: vanilla PPO loss + entropy + KL, forward and backward (dp_actor.py:419-466)
# --------------------------------------------------------------------------------------------
def ppo_loss_inputs(g, B, R, kind):
    old = -torch.rand(B, R, generator=g) * 6.0
    delta = torch.randn(B, R, generator=g) * 0.3
    if kind == "edges":
        # hit the +-20 clamp, exact clip bounds and exact ties
        delta[0, :4] = torch.tensor([25.0, -25.0, 20.0, -20.0])
        delta[1, :3] = torch.tensor([float(np.log(np.float32(1.2))), float(np.log(np.float32(0.8))), 0.0])
    logp = old + delta
    adv = torch.randn(B, R, generator=g)
    if kind == "edges":
        adv[:, 5] = 0.0
        adv[2, :] = -adv[2, :].abs()  # a row of negative advantages (dual-clip path)
    mask = torch.ones(B, R, dtype=torch.int64)
    lengths = torch.randint(1, R + 1, (B,), generator=g)
    for i in range(B):
        mask[i, lengths[i]:] = 0
    if kind == "edges" and B > 3:
        mask[3, :] = 0  # fully masked row
        mask[3, 0] = 1
    ent = torch.rand(B, R, generator=g) * 3.0
    ref = logp + torch.randn(B, R, generator=g) * 0.2
    if kind == "edges":
        ref[0, 6:8] = logp[0, 6:8] + torch.tensor([30.0, -30.0])  # k3 clamps
    return old.float(), logp.float(), adv.float(), mask, ent.float(), ref.float()


def ref_actor_loss(old, logp, adv, mask, ent, ref, cfg):
    logp = logp.clone().requires_grad_(True)
    ent = ent.clone().requires_grad_(True)
    pcfg = DictConfig(
        clip_ratio=cfg["clip_ratio"],
        clip_ratio_low=cfg["clip_ratio_low"],
        clip_ratio_high=cfg["clip_ratio_high"],
        clip_ratio_c=cfg["clip_ratio_c"],
    )
    mode = cfg["loss_agg_mode"]
    pg_loss, pg_clipfrac, ppo_kl, pg_clipfrac_lower = ca.compute_policy_loss_vanilla(
        old_log_prob=old, log_prob=logp, advantages=adv, response_mask=mask, loss_agg_mode=mode, config=pcfg
    )
    entropy_loss = ca.agg_loss(loss_mat=ent, loss_mask=mask, loss_agg_mode=mode)
    policy_loss = pg_loss - entropy_loss * cfg["entropy_coeff"] if cfg["entropy_coeff"] != 0 else pg_loss
    kld = ca.kl_penalty(logprob=logp, ref_logprob=ref, kl_penalty=cfg["kl_loss_type"])
    kl_loss = ca.agg_loss(loss_mat=kld, loss_mask=mask, loss_agg_mode=mode)
    if cfg["use_kl_loss"]:
        policy_loss = policy_loss + kl_loss * cfg["kl_loss_coef"]
    loss = policy_loss * cfg["loss_scale_factor"]
    loss.backward()
    return dict(
        pg_loss=pg_loss.detach(),
        pg_clipfrac=pg_clipfrac.detach(),
        ppo_kl=ppo_kl.detach(),
        pg_clipfrac_lower=pg_clipfrac_lower.detach(),
        entropy_loss=entropy_loss.detach(),
        kl_loss=kl_loss.detach(),
        loss=loss.detach(),
        dlogp=logp.grad.detach() if logp.grad is not None else torch.zeros_like(logp),
        dentropy=ent.grad.detach() if ent.grad is not None else torch.zeros_like(ent),
        kld=kld.detach(),
    )


def gen_ppo_loss():
    g = torch.Generator().manual_seed(1234)
    arrays, cases = {}, []
    modes = ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"]
    kls = ["low_var_kl", "kl", "abs", "mse", "k3", "k1", "k2"]
    ci = 0
    for shape, kind in [((6, 16), "edges"), ((8, 64), "random"), ((16, 256), "random"), ((5, 33), "edges")]:
        for mode in modes:
            for kl in ([kls[ci % len(kls)], "low_var_kl"] if shape != (6, 16) else kls):
                cfg = dict(
                    clip_ratio=0.2,
                    clip_ratio_low=0.2,
                    clip_ratio_high=0.28 if ci % 3 == 1 else 0.2,
                    clip_ratio_c=10.0 if ci % 3 == 1 else 3.0,
                    loss_agg_mode=mode,
                    entropy_coeff=[0.0, 0.001, 0.01][ci % 3],
                    use_kl_loss=ci % 4 != 3,
                    kl_loss_type=kl,
                    kl_loss_coef=0.001 if ci % 2 == 0 else 0.05,
                    loss_scale_factor=[1.0, 0.5, 0.125][ci % 3],
                )
                ins = ppo_loss_inputs(g, *shape, kind)
                outs = ref_actor_loss(*ins, cfg)
                for k, v in zip(["old_log_prob", "log_prob", "advantages", "response_mask", "entropy", "ref_log_prob"], ins):
                    arrays[f"c{ci}_{k}"] = v
                for k, v in outs.items():
                    arrays[f"c{ci}_out_{k}"] = v
                cases.append(cfg)
                ci += 1
    _save("ppo_loss.npz", arrays, {"cases": cases, "ref": "core_algos.py:703-889,1272-1307; dp_actor.py:419-466"})


# --------------------------------------------------------------------------------------------
# A11: masked_mean known answers from the reference's own test (tests/utils/test_torch_functional.py:55-66)
# --------------------------------------------------------------------------------------------
def gen_masked_mean():
    arrays = {}
    vals = torch.tensor([1.0, 2.0, float("nan"), 4.0])
    mask = torch.tensor([1.0, 1.0, 0.0, 1.0])
    arrays["kat_values"] = vals
    arrays["kat_mask"] = mask
    arrays["kat_out"] = vF.masked_mean(vals, mask)
    g = torch.Generator().manual_seed(7)
    v = torch.randn(9, 37, generator=g)
    m = (torch.rand(9, 37, generator=g) > 0.3).to(torch.int64)
    arrays["rand_values"] = v
    arrays["rand_mask"] = m
    arrays["rand_out_all"] = vF.masked_mean(v, m)
    arrays["rand_out_axis1"] = vF.masked_mean(v, m, axis=1)
    arrays["rand_whiten"] = vF.masked_whiten(v, m)
    arrays["rand_var"] = vF.masked_var(v, m)
    _save("masked_mean.npz", arrays, {"ref": "torch_functional.py:163-223; tests/utils/test_torch_functional.py:55-66"})


# --------------------------------------------------------------------------------------------
# A17: GRPO outcome advantage (core_algos.py:260-324)
# --------------------------------------------------------------------------------------------
def gen_grpo():
    g = torch.Generator().manual_seed(99)
    arrays, cases = {}, []
    layouts = [
        ("n8_interleaved", [8] * 8, False),
        ("ragged_with_singletons", [3, 1, 5, 1, 2, 4], True),
        ("n8_shuffled", [8] * 6, True),
        ("ties_zero_std", [4, 4], False),
    ]
    ci = 0
    for name, sizes, shuffle in layouts:
        B = sum(sizes)
        R = 24
        uid = np.concatenate([np.full(s, f"uid-{gi}", dtype=object) for gi, s in enumerate(sizes)])
        if shuffle:
            perm = torch.randperm(B, generator=g).numpy()
            uid = uid[perm]
        mask = torch.ones(B, R, dtype=torch.int64)
        lengths = torch.randint(1, R + 1, (B,), generator=g)
        for i in range(B):
            mask[i, lengths[i]:] = 0
        rewards = torch.zeros(B, R)
        if name == "ties_zero_std":
            score = torch.ones(B)
        else:
            score = torch.bernoulli(torch.full((B,), 0.5), generator=g) + torch.randn(B, generator=g) * 0.1
        for i in range(B):
            rewards[i, lengths[i] - 1] = score[i]
        if ci == 1:
            rewards += torch.randn(B, R, generator=g) * 0.01 * mask  # dense token rewards too
        for norm in (True, False):
            adv, ret = ca.compute_grpo_outcome_advantage(
                token_level_rewards=rewards, response_mask=mask, index=uid, norm_adv_by_std_in_grpo=norm
            )
            arrays[f"c{ci}_rewards"] = rewards
            arrays[f"c{ci}_mask"] = mask
            arrays[f"c{ci}_uid"] = np.array([str(u) for u in uid])
            arrays[f"c{ci}_adv"] = adv
            arrays[f"c{ci}_ret"] = ret
            cases.append({"name": name, "norm_adv_by_std_in_grpo": norm, "epsilon": 1e-6})
            ci += 1
    _save("grpo.npz", arrays, {"cases": cases, "ref": "core_algos.py:260-324"})


# --------------------------------------------------------------------------------------------
# A18: GAE + masked_whiten (core_algos.py:208-256)
# --------------------------------------------------------------------------------------------
def gen_gae():
    g = torch.Generator().manual_seed(5)
    arrays, cases = {}, []
    for ci, (B, R, gamma, lam, obs) in enumerate([(4, 12, 1.0, 1.0, False), (8, 64, 0.99, 0.95, True), (3, 7, 0.9, 0.5, True)]):
        rewards = torch.randn(B, R, generator=g)
        values = torch.randn(B, R, generator=g)
        mask = torch.ones(B, R, dtype=torch.int64)
        lengths = torch.randint(2, R + 1, (B,), generator=g)
        for i in range(B):
            mask[i, lengths[i]:] = 0
        if obs:  # observation tokens inside the response (multi-turn), test_core_algos_on_cpu.py:134-188
            mask[:, 1] = 0
        adv, ret = ca.compute_gae_advantage_return(rewards, values, mask, gamma=gamma, lam=lam)
        arrays[f"c{ci}_rewards"] = rewards
        arrays[f"c{ci}_values"] = values
        arrays[f"c{ci}_mask"] = mask
        arrays[f"c{ci}_adv"] = adv
        arrays[f"c{ci}_ret"] = ret
        cases.append({"gamma": gamma, "lam": lam})
    _save("gae.npz", arrays, {"cases": cases, "ref": "core_algos.py:208-256; torch_functional.py:206-223"})


# --------------------------------------------------------------------------------------------
# A8/A9: log-prob + entropy over the vocabulary, forward and backward (torch_functional.py:116-160)
# --------------------------------------------------------------------------------------------
def seeded_logits(seed, N, V, scale=3.0):
    rng = np.random.default_rng(seed)
    x = (rng.standard_normal((N, V), dtype=np.float32) * np.float32(scale)).astype(np.float32)
    labels = rng.integers(0, V, size=(N,), dtype=np.int64)
    dlogp = rng.standard_normal((N,), dtype=np.float32)
    dent = rng.standard_normal((N,), dtype=np.float32)
    return x, labels, dlogp, dent


def gen_logprob():
    arrays, cases = {}, []
    specs = [(11, 64, 1000, False), (12, 33, 4099, False), (13, 8, 151936, True), (14, 17, 151936, True)]
    for ci, (seed, N, V, from_seed) in enumerate(specs):
        x, labels, dlogp, dent = seeded_logits(seed, N, V)
        for dt in ("fp32", "bf16"):
            logits = torch.from_numpy(x)
            if dt == "bf16":
                logits = logits.to(torch.bfloat16)
            # fp32 path of the reference (flash-attn CE semantics = fp32 math on the given logits)
            lf = logits.float().clone().requires_grad_(True)
            lp = vF.logprobs_from_logits_v2(lf, torch.from_numpy(labels))
            ent = vF.entropy_from_logits(lf)
            (lp * torch.from_numpy(dlogp)).sum().backward(retain_graph=True)
            g_lp = lf.grad.clone()
            lf.grad = None
            (ent * torch.from_numpy(dent)).sum().backward()
            g_ent = lf.grad.clone()
            key = f"c{ci}_{dt}"
            arrays[f"{key}_logp"] = lp.detach()
            arrays[f"{key}_entropy"] = ent.detach()
            # backward outputs are large at V=151936; keep checksums + a strided sample there
            if from_seed:
                idx = np.arange(0, N * V, 997)
                arrays[f"{key}_dlogits_lp_sample"] = g_lp.reshape(-1)[idx]
                arrays[f"{key}_dlogits_ent_sample"] = g_ent.reshape(-1)[idx]
                arrays[f"{key}_dlogits_lp_rowsum_abs"] = g_lp.abs().sum(-1)
                arrays[f"{key}_dlogits_ent_rowsum_abs"] = g_ent.abs().sum(-1)
            else:
                arrays[f"{key}_dlogits_lp"] = g_lp
                arrays[f"{key}_dlogits_ent"] = g_ent
            if dt == "bf16":
                # the reference's own bf16 path (keeps bf16 output, torch_functional.py:125-133)
                arrays[f"{key}_logp_refbf16"] = vF.logprobs_from_logits_v2(logits, torch.from_numpy(labels)).float()
        if not from_seed:
            arrays[f"c{ci}_logits"] = x
            arrays[f"c{ci}_labels"] = labels
            arrays[f"c{ci}_dlogp"] = dlogp
            arrays[f"c{ci}_dentropy"] = dent
        arrays[f"c{ci}_sha256"] = np.array(hashlib.sha256(x.tobytes()).hexdigest())
        cases.append({"seed": seed, "N": N, "V": V, "inputs_from_seed": from_seed, "scale": 3.0})
    _save("logprob.npz", arrays, {"cases": cases, "generator": "numpy default_rng(seed): standard_normal(N,V,f32)*scale, integers(0,V,N), standard_normal(N) x2",
                                  "ref": "torch_functional.py:116-160"})


# --------------------------------------------------------------------------------------------
# A21: FusedLinearForPPO (utils/experimental/torch_functional.py:20-216)
# --------------------------------------------------------------------------------------------
def gen_fused_linear():
    arrays, cases = {}, []
    for ci, (seed, N, H, V, temp) in enumerate([(21, 40, 64, 512, 1.0), (22, 130, 96, 1000, 1.5)]):
        rng = np.random.default_rng(seed)
        h = (rng.random((N, H), dtype=np.float32) - 0.5).astype(np.float32)
        w = (rng.random((V, H), dtype=np.float32) - 0.5).astype(np.float32)
        ids = rng.integers(0, V, size=(N,), dtype=np.int64)
        dlp = rng.standard_normal((N,), dtype=np.float32)
        den = rng.standard_normal((N,), dtype=np.float32)
        ht = torch.from_numpy(h).requires_grad_(True)
        wt = torch.from_numpy(w).requires_grad_(True)
        lp, ent = vxf.FusedLinearForPPO(chunk_size=32)(ht, wt, torch.from_numpy(ids), temperature=temp)
        ((lp * torch.from_numpy(dlp)).sum() + (ent * torch.from_numpy(den)).sum()).backward()
        for k, v in dict(hidden=h, weight=w, input_ids=ids, dlogp=dlp, dentropy=den, out_logp=lp.detach(),
                         out_entropy=ent.detach(), out_dhidden=ht.grad, out_dweight=wt.grad).items():
            arrays[f"c{ci}_{k}"] = v
        cases.append({"N": N, "H": H, "V": V, "temperature": temp})
    _save("fused_linear.npz", arrays, {"cases": cases, "ref": "utils/experimental/torch_functional.py:20-216"})


# --------------------------------------------------------------------------------------------
# A4/A5: response mask, prompt positions and response-position continuation
# --------------------------------------------------------------------------------------------
def gen_masks():
    arrays = {}
    # the docstring example of get_response_mask (torch_functional.py:226-246)
    resp = torch.tensor([[20, 10, 34, 1, 0, 0, 0], [78, 0, 76, 2, 1, 0, 0], [23, 98, 1, 0, 0, 0, 0], [33, 3, 98, 45, 1, 0, 0]])
    arrays["doc_responses"] = resp
    arrays["doc_mask_eos1"] = vF.get_response_mask(resp, eos_token=1)
    arrays["doc_mask_eos12"] = vF.get_response_mask(resp, eos_token=[1, 2])
    g = torch.Generator().manual_seed(3)
    r = torch.randint(0, 40, (32, 50), generator=g)
    r[5, :] = 7  # row that is all EOS
    arrays["rand_responses"] = r
    arrays["rand_mask_eos7"] = vF.get_response_mask(r, eos_token=7)
    arrays["rand_mask_eos7_9_11"] = vF.get_response_mask(r, eos_token=[7, 9, 11])
    # left-padded prompt attention masks -> position ids (utils/model.py:219)
    am = torch.ones(16, 20, dtype=torch.int64)
    pads = torch.randint(0, 20, (16,), generator=g)
    for i in range(16):
        am[i, : pads[i]] = 0
    arrays["prompt_attention_mask"] = am
    pos = compute_position_id_with_mask(am)
    arrays["prompt_position_ids"] = pos
    # response position continuation (hf_rollout.py:151-155)
    R = 9
    delta = torch.arange(1, R + 1).unsqueeze(0).repeat(16, 1)
    arrays["full_position_ids"] = torch.cat([pos, pos[:, -1:] + delta], dim=-1)
    _save("masks.npz", arrays, {"ref": "torch_functional.py:226-246; model.py:219; hf_rollout.py:151-160"})


# --------------------------------------------------------------------------------------------
# A3/A6: tiny random Qwen2 — HF greedy generate post-processed exactly as HFRollout._generate_minibatch
# (hf_rollout.py:112-171), and teacher-forced log-probs / entropy of the responses as
# DataParallelPPOActor._forward_micro_batch computes them (dp_actor.py:249-272), all fp32.
# --------------------------------------------------------------------------------------------
TINY_QWEN2 = dict(vocab_size=512, hidden_size=64, intermediate_size=128, num_hidden_layers=2, num_attention_heads=4,
                  num_key_value_heads=2, max_position_embeddings=256, rope_theta=10000.0, rms_norm_eps=1e-6,
                  tie_word_embeddings=True, initializer_range=0.2, bos_token_id=1, eos_token_id=2, pad_token_id=0)


def gen_tiny_qwen2():
    from safetensors.torch import save_file
    from transformers import GenerationConfig, Qwen2Config, Qwen2ForCausalLM

    torch.manual_seed(0)
    cfg = Qwen2Config(**TINY_QWEN2, attn_implementation="eager")
    model = Qwen2ForCausalLM(cfg).float().eval()
    with torch.no_grad():  # non-trivial norm weights and biases so those code paths are exercised
        for n, p in model.named_parameters():
            if "norm" in n:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
            elif n.endswith("bias"):
                p.copy_(0.1 * torch.randn_like(p))
    outdir = os.path.join(HERE, "tiny_qwen2")
    os.makedirs(outdir, exist_ok=True)
    sd = {k: v.contiguous() for k, v in model.state_dict().items() if k != "lm_head.weight"}
    save_file(sd, os.path.join(outdir, "model.safetensors"))
    with open(os.path.join(outdir, "config.json"), "w") as f:
        json.dump(TINY_QWEN2, f, indent=1)

    B, P, R = 6, 12, 10
    g = torch.Generator().manual_seed(42)
    ids = torch.randint(3, 512, (B, P), generator=g)
    am = torch.ones(B, P, dtype=torch.int64)
    for i, npad in enumerate([0, 3, 0, 5, 1, 0]):
        am[i, :npad] = 0
        ids[i, :npad] = TINY_QWEN2["pad_token_id"]
    pos = compute_position_id_with_mask(am)

    def hf_rollout(eos):
        gc = GenerationConfig(do_sample=False, num_beams=1)
        with torch.no_grad():
            out = model.generate(input_ids=ids, attention_mask=am, do_sample=False, max_new_tokens=R,
                                 eos_token_id=eos, pad_token_id=TINY_QWEN2["pad_token_id"], generation_config=gc,
                                 output_scores=True, return_dict_in_generate=True, use_cache=True)
        seq = out.sequences
        if seq.shape[1] < P + R:  # hf_rollout.py:132-139
            seq = torch.cat([seq, torch.full((B, P + R - seq.shape[1]), TINY_QWEN2["pad_token_id"])], 1)
        gaps = [torch.topk(s, 2, dim=-1).values for s in out.scores]
        gap = min(float((v[:, 0] - v[:, 1]).min()) for v in gaps)
        return seq, gap

    seq, gap = hf_rollout(eos=[TINY_QWEN2["eos_token_id"]])
    eos = int(seq[0, P + 4])  # make row 0 hit "EOS" mid-response so the finished-row padding path is exercised
    seq, gap = hf_rollout(eos=[eos])
    resp = seq[:, P:]
    delta = torch.arange(1, R + 1).unsqueeze(0).repeat(B, 1)
    full_pos = torch.cat([pos, pos[:, -1:] + delta], -1)
    resp_mask = vF.get_response_mask(resp, eos_token=eos, dtype=am.dtype)
    full_am = torch.cat([am, resp_mask], -1)
    with torch.no_grad():
        logits = model(input_ids=seq, attention_mask=full_am, position_ids=full_pos, use_cache=False).logits
    logits = logits[:, -R - 1:-1, :]
    logp = vF.logprobs_from_logits_v2(logits, resp)
    ent = vF.entropy_from_logits(logits)
    # temperature 0.7 variant (logits.div_(temperature), dp_actor.py:263)
    logp_t = vF.logprobs_from_logits_v2(logits / 0.7, resp)
    arrays = dict(prompt_ids=ids, prompt_attention_mask=am, prompt_position_ids=pos, sequences=seq,
                  responses=resp, attention_mask=full_am, position_ids=full_pos, log_probs=logp, entropy=ent,
                  log_probs_t07=logp_t)
    _save("tiny_qwen2_rollout.npz", arrays, {"eos_token_id": eos, "pad_token_id": TINY_QWEN2["pad_token_id"],
                                             "response_length": R, "min_top2_logit_gap": gap,
                                             "hf": "transformers Qwen2ForCausalLM fp32 eager attention",
                                             "ref": "hf_rollout.py:112-171; dp_actor.py:249-272"})


# --------------------------------------------------------------------------------------------
# K6: critic clipped value loss + backward (core_algos.py:1230-1269; dp_critic.py:218-245)
# --------------------------------------------------------------------------------------------
def gen_value_loss():
    g = torch.Generator().manual_seed(11)
    arrays, cases = {}, []
    ci = 0
    for dt in ["float32", "bfloat16"]:
        for mode in ["token-mean", "seq-mean-token-sum", "seq-mean-token-mean", "seq-mean-token-sum-norm"]:
            for clip, lsf in [(0.5, 0.25), (0.2, 1.0)]:
                B, R = (6, 40) if ci % 2 == 0 else (3, 129)
                values = torch.randn(B, R, generator=g) * 0.8
                vpreds = values + torch.randn(B, R, generator=g) * 0.6
                returns = values + torch.randn(B, R, generator=g)
                mask = torch.ones(B, R, dtype=torch.int64)
                for i in range(B):
                    mask[i, int(torch.randint(1, R + 1, (1,), generator=g)):] = 0
                tdt = getattr(torch, dt)
                values, vpreds = values.to(tdt), vpreds.to(tdt)
                # edges: vpred exactly on the clip bounds (ties in torch.min / torch.max), vpred == value
                vpreds[0, 0] = (values[0, 0] + clip).to(tdt)
                vpreds[0, 1] = (values[0, 1] - clip).to(tdt)
                vpreds[0, 2] = values[0, 2]
                returns[0, 3] = vpreds[0, 3].float()  # zero error
                vp = vpreds.clone().requires_grad_(True)
                vf_loss, vf_clipfrac = ca.compute_value_loss(vpreds=vp, returns=returns, values=values,
                                                             response_mask=mask, cliprange_value=clip,
                                                             loss_agg_mode=mode)
                (vf_loss * lsf).backward()
                vpred_mean = vF.masked_mean(vpreds, mask)
                for k, v in dict(vpreds=vpreds, values=values, returns=returns, mask=mask, vf_loss=vf_loss.detach(),
                                 vf_clipfrac=vf_clipfrac.detach(), vpred_mean=vpred_mean.detach(),
                                 dvpreds=vp.grad).items():
                    arrays[f"c{ci}_{k}"] = v.float() if torch.is_tensor(v) and v.is_floating_point() else v
                cases.append({"dtype": dt, "mode": mode, "cliprange_value": clip, "loss_scale_factor": lsf})
                ci += 1
    _save("value_loss.npz", arrays, {"cases": cases, "ref": "core_algos.py:1230-1269; dp_critic.py:218-245"})


def gen_gae_bf16():
    """GAE over bf16 critic values (the dtype dp_critic.compute_values returns under autocast)."""
    g = torch.Generator().manual_seed(6)
    arrays, cases = {}, []
    for ci, (B, R, gamma, lam) in enumerate([(5, 33, 0.99, 0.95), (4, 16, 1.0, 0.9)]):
        rewards = torch.randn(B, R, generator=g)
        values = torch.randn(B, R, generator=g).to(torch.bfloat16)
        mask = torch.ones(B, R, dtype=torch.int64)
        for i in range(B):
            mask[i, int(torch.randint(2, R + 1, (1,), generator=g)):] = 0
        adv, ret = ca.compute_gae_advantage_return(rewards, values, mask, gamma=gamma, lam=lam)
        arrays.update({f"c{ci}_rewards": rewards, f"c{ci}_values": values.float(), f"c{ci}_mask": mask,
                       f"c{ci}_adv": adv, f"c{ci}_ret": ret})
        cases.append({"gamma": gamma, "lam": lam})
    _save("gae_bf16.npz", arrays, {"cases": cases, "values_dtype": "bfloat16", "ref": "core_algos.py:208-256"})


def gen_tiny_critic():
    """Critic = the tiny backbone + a `score` head (Qwen2ForTokenClassification, num_labels=1, dropout 0, as
    fsdp_workers.py:1045-1056 configures it), fp32: values over the tiny rollout sequences (dp_critic.py:127-145
    padded path), then one micro-batch value loss (token-mean, cliprange 0.5, loss_scale_factor 0.5) and its
    backward; records values and the gradients of the head, the final norm and the first layer norm."""
    from safetensors.torch import load_file, save_file
    from transformers import Qwen2Config, Qwen2ForTokenClassification

    cfg = Qwen2Config(**TINY_QWEN2, attn_implementation="eager", num_labels=1, classifier_dropout=0.0)
    model = Qwen2ForTokenClassification(cfg).float()
    sd = load_file(os.path.join(HERE, "tiny_qwen2", "model.safetensors"))
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert set(missing) == {"score.weight", "score.bias"} and not unexpected, (missing, unexpected)
    g = torch.Generator().manual_seed(77)
    with torch.no_grad():
        model.score.weight.copy_(torch.randn(model.score.weight.shape, generator=g) * 0.2)
        model.score.bias.copy_(torch.randn(1, generator=g) * 0.1)
    save_file({"score.weight": model.score.weight.detach().contiguous(), "score.bias": model.score.bias.detach()},
              os.path.join(HERE, "tiny_qwen2", "score.safetensors"))
    z = np.load(os.path.join(HERE, "tiny_qwen2_rollout.npz"))
    seq, am, pos = (torch.from_numpy(z[k]) for k in ("sequences", "attention_mask", "position_ids"))
    resp = torch.from_numpy(z["responses"])
    R = resp.shape[1]
    rmask = am[:, -R:]
    model.train()
    vpreds = model(input_ids=seq, attention_mask=am, position_ids=pos, use_cache=False).logits
    vpreds = vpreds[:, -R - 1:-1].squeeze(-1)
    values = (vpreds.detach() + 0.3 * torch.randn(vpreds.shape, generator=g)) * rmask
    returns = values + torch.randn(vpreds.shape, generator=g)
    vf_loss, vf_clipfrac = ca.compute_value_loss(vpreds=vpreds, returns=returns, values=values, response_mask=rmask,
                                                 cliprange_value=0.5, loss_agg_mode="token-mean")
    (vf_loss * 0.5).backward()
    arrays = dict(vpreds=vpreds.detach(), values=values, returns=returns, vf_loss=vf_loss.detach(),
                  vf_clipfrac=vf_clipfrac, d_score_weight=model.score.weight.grad, d_score_bias=model.score.bias.grad,
                  d_norm=model.model.norm.weight.grad,
                  d_input_layernorm0=model.model.layers[0].input_layernorm.weight.grad,
                  d_embed_rows=model.model.embed_tokens.weight.grad.norm(dim=-1))
    _save("tiny_critic.npz", arrays, {"cliprange_value": 0.5, "loss_agg_mode": "token-mean", "loss_scale_factor": 0.5,
                                      "hf": "transformers Qwen2ForTokenClassification fp32 eager attention",
                                      "ref": "dp_critic.py:127-145, 218-245; core_algos.py:1230-1269"})


# --------------------------------------------------------------------------------------------
# DAPO overlong-buffer reward (reward_manager/dapo.py:60-150) with a stub tokenizer / scorer
# --------------------------------------------------------------------------------------------
def gen_dapo_reward():
    from verl import DataProto as RefDataProto
    from verl.workers.reward_manager.dapo import DAPORewardManager

    class Tok:
        eos_token = "</s>"

        def decode(self, ids, skip_special_tokens=True):
            return ",".join(str(int(i)) for i in ids)

    g = torch.Generator().manual_seed(9)
    arrays, cases = {}, []
    for ci, (B, P, R, blen, factor) in enumerate([(6, 4, 12, 4, 1.5), (16, 8, 64, 16, 1.0)]):
        prompts = torch.randint(3, 100, (B, P), generator=g)
        resp = torch.randint(3, 100, (B, R), generator=g)
        lens = torch.randint(0, R + 1, (B,), generator=g)
        lens[0], lens[1] = R, 0
        am = torch.ones(B, P + R, dtype=torch.int64)
        for i in range(B):
            am[i, P + int(lens[i]):] = 0
        acc = (torch.rand(B, generator=g) > 0.5).float()
        table = {",".join(str(int(t)) for t in resp[i, : int(lens[i])]): float(acc[i]) for i in range(B)}
        ob = DictConfig(enable=True, len=blen, penalty_factor=factor, log=True)
        rm = DAPORewardManager(Tok(), num_examine=0, compute_score=lambda data_source, solution_str, ground_truth,
                               extra_info=None: table[solution_str], max_resp_len=R, overlong_buffer_cfg=ob)
        dp = RefDataProto.from_dict(tensors={"prompts": prompts, "responses": resp, "attention_mask": am},
                                    non_tensors={"reward_model": np.array([{"ground_truth": ""}] * B, dtype=object),
                                                 "data_source": np.array(["synthetic"] * B, dtype=object)})
        out = rm(dp, return_dict=True)
        over = np.array([float(x) for x in out["reward_extra_info"]["overlong_reward"]], np.float32)
        arrays.update({f"c{ci}_responses": resp, f"c{ci}_attention_mask": am, f"c{ci}_acc": acc,
                       f"c{ci}_reward_tensor": out["reward_tensor"], f"c{ci}_overlong_reward": over})
        cases.append({"max_resp_len": R, "overlong_len": blen, "penalty_factor": factor})
    _save("dapo_reward.npz", arrays, {"cases": cases, "ref": "reward_manager/dapo.py:60-150"})


# --------------------------------------------------------------------------------------------
# Llama family (config #4's Llama-3-8B architecture: no q/k/v bias, untied lm_head, head_dim 128,
# rope_theta 5e5): tiny LlamaForCausalLM greedy rollout + teacher-forced log-probs (fp32, eager)
# --------------------------------------------------------------------------------------------
TINY_LLAMA = dict(vocab_size=512, hidden_size=256, intermediate_size=256, num_hidden_layers=2, num_attention_heads=2,
                  num_key_value_heads=1, max_position_embeddings=256, rope_theta=500000.0, rms_norm_eps=1e-5,
                  tie_word_embeddings=False, initializer_range=0.1, bos_token_id=1, eos_token_id=2, pad_token_id=0,
                  attention_bias=False, mlp_bias=False, model_type="llama")


def gen_tiny_llama():
    from safetensors.torch import save_file
    from transformers import GenerationConfig, LlamaConfig, LlamaForCausalLM

    torch.manual_seed(1)
    kw = {k: v for k, v in TINY_LLAMA.items() if k != "model_type"}
    cfg = LlamaConfig(**kw, attn_implementation="eager")
    model = LlamaForCausalLM(cfg).float().eval()
    with torch.no_grad():
        for n, p in model.named_parameters():
            if "norm" in n:
                p.copy_(1.0 + 0.1 * torch.randn_like(p))
    outdir = os.path.join(HERE, "tiny_llama")
    os.makedirs(outdir, exist_ok=True)
    save_file({k: v.contiguous() for k, v in model.state_dict().items()}, os.path.join(outdir, "model.safetensors"))
    with open(os.path.join(outdir, "config.json"), "w") as f:
        json.dump(TINY_LLAMA, f, indent=1)
    B, P, R = 4, 10, 8
    g = torch.Generator().manual_seed(43)
    ids = torch.randint(3, 512, (B, P), generator=g)
    am = torch.ones(B, P, dtype=torch.int64)
    for i, npad in enumerate([0, 2, 0, 4]):
        am[i, :npad] = 0
        ids[i, :npad] = TINY_LLAMA["pad_token_id"]
    pos = compute_position_id_with_mask(am)
    gc = GenerationConfig(do_sample=False, num_beams=1)
    with torch.no_grad():
        out = model.generate(input_ids=ids, attention_mask=am, do_sample=False, max_new_tokens=R, eos_token_id=[2],
                             pad_token_id=0, generation_config=gc, output_scores=True, return_dict_in_generate=True,
                             use_cache=True)
    seq = out.sequences
    if seq.shape[1] < P + R:
        seq = torch.cat([seq, torch.zeros(B, P + R - seq.shape[1], dtype=seq.dtype)], 1)
    gap = min(float((v[:, 0] - v[:, 1]).min()) for v in (torch.topk(s_, 2, dim=-1).values for s_ in out.scores))
    resp = seq[:, P:]
    full_pos = torch.cat([pos, pos[:, -1:] + torch.arange(1, R + 1).unsqueeze(0).repeat(B, 1)], -1)
    resp_mask = vF.get_response_mask(resp, eos_token=2, dtype=am.dtype)
    full_am = torch.cat([am, resp_mask], -1)
    with torch.no_grad():
        logits = model(input_ids=seq, attention_mask=full_am, position_ids=full_pos, use_cache=False).logits
    logits = logits[:, -R - 1:-1, :]
    arrays = dict(prompt_ids=ids, prompt_attention_mask=am, prompt_position_ids=pos, sequences=seq, responses=resp,
                  attention_mask=full_am, position_ids=full_pos, log_probs=vF.logprobs_from_logits_v2(logits, resp),
                  entropy=vF.entropy_from_logits(logits))
    _save("tiny_llama_rollout.npz", arrays, {"eos_token_id": 2, "pad_token_id": 0, "response_length": R,
                                             "min_top2_logit_gap": gap,
                                             "hf": "transformers LlamaForCausalLM fp32 eager attention",
                                             "ref": "hf_rollout.py:112-171; dp_actor.py:249-272"})


# --------------------------------------------------------------------------------------------
# sequence-length balancing (utils/seqlen_balancing.py:26-239): Karmarkar-Karp partitions used by
# trainer.balance_batch (equal_size) and dynamic micro-batching (unequal), + the imbalance metrics
# --------------------------------------------------------------------------------------------
def gen_seqlen():
    from verl.utils import seqlen_balancing as sb

    rng = np.random.default_rng(21)
    cases = []
    for ci, (B, k, eq) in enumerate([(16, 4, True), (64, 8, True), (512, 8, True), (37, 5, False), (64, 7, False),
                                     (128, 3, False), (8, 8, True), (12, 1, False)]):
        lens = [int(x) for x in rng.integers(64, 768, size=B)]
        if ci == 1:
            lens[:10] = [500] * 10  # ties
        parts = sb.get_seqlen_balanced_partitions(lens, k_partitions=k, equal_size=eq)
        stats = sb.log_seqlen_unbalance(seqlen_list=lens, partitions=parts, prefix="global_seqlen") if eq else {}
        cases.append({"seqlens": lens, "k": k, "equal_size": eq, "partitions": parts,
                      "stats": {kk: float(v) for kk, v in stats.items()}})
    path = os.path.join(HERE, "seqlen_balancing.json")
    with open(path, "w") as f:
        json.dump({"cases": cases, "ref": "utils/seqlen_balancing.py:26-239"}, f)
    print(f"wrote {path} ({os.path.getsize(path)} bytes)")


# --------------------------------------------------------------------------------------------
# RLOO (core_algos.py:444-493) and REINFORCE++-baseline (core_algos.py:392-441) on the GRPO layouts
# --------------------------------------------------------------------------------------------
def gen_group_adv():
    g = torch.Generator().manual_seed(101)
    arrays, cases = {}, []
    ci = 0
    for name, sizes, shuffle in [("n8_interleaved", [8] * 8, False), ("ragged_with_singletons", [3, 1, 5, 1, 2, 4], True),
                                 ("n4_shuffled", [4] * 6, True)]:
        B, R = sum(sizes), 20
        uid = np.concatenate([np.full(s, f"uid-{gi}", dtype=object) for gi, s in enumerate(sizes)])
        if shuffle:
            uid = uid[torch.randperm(B, generator=g).numpy()]
        mask = torch.ones(B, R, dtype=torch.int64)
        lengths = torch.randint(2, R + 1, (B,), generator=g)
        for i in range(B):
            mask[i, lengths[i]:] = 0
        rewards = torch.zeros(B, R)
        score = torch.bernoulli(torch.full((B,), 0.5), generator=g) + torch.randn(B, generator=g) * 0.1
        for i in range(B):
            rewards[i, lengths[i] - 1] = score[i]
        for est, fn in [("rloo", ca.compute_rloo_outcome_advantage),
                        ("reinforce_plus_plus_baseline", ca.compute_reinforce_plus_plus_baseline_outcome_advantage)]:
            adv, ret = fn(token_level_rewards=rewards.clone(), response_mask=mask, index=uid)
            arrays.update({f"c{ci}_rewards": rewards, f"c{ci}_mask": mask, f"c{ci}_uid": np.array([str(u) for u in uid]),
                           f"c{ci}_adv": adv, f"c{ci}_ret": ret})
            cases.append({"name": name, "estimator": est})
            ci += 1
    _save("group_adv.npz", arrays, {"cases": cases, "ref": "core_algos.py:392-493"})


def gen_more_adv():
    """OPO (core_algos.py:495-546), GPG (:624-684), GRPO pass@k (:327-386) on uid-group layouts, and ReMax
    (:588-621) with per-row baselines."""
    g = torch.Generator().manual_seed(107)
    arrays, cases = {}, []
    ci = 0
    for name, sizes, shuffle in [("n8_interleaved", [8] * 8, False), ("ragged", [3, 2, 5, 2, 4], True),
                                 ("n4_shuffled", [4] * 6, True), ("with_singletons", [3, 1, 4, 1, 2], True)]:
        B, R = sum(sizes), 20
        uid = np.concatenate([np.full(s, f"uid-{gi}", dtype=object) for gi, s in enumerate(sizes)])
        if shuffle:
            uid = uid[torch.randperm(B, generator=g).numpy()]
        mask = torch.ones(B, R, dtype=torch.int64)
        lengths = torch.randint(2, R + 1, (B,), generator=g)
        for i in range(B):
            mask[i, lengths[i]:] = 0
        rewards = torch.zeros(B, R)
        score = torch.bernoulli(torch.full((B,), 0.5), generator=g) + torch.randn(B, generator=g) * 0.1
        score[::3] = torch.round(score[::3]).clamp(0, 1)  # exact 0 / 1 scores: GPG's nonzero count, pass@k ties
        for i in range(B):
            rewards[i, lengths[i] - 1] = score[i]
        ests = [("opo", lambda r, m, u: ca.compute_opo_outcome_advantage(token_level_rewards=r, response_mask=m, index=u)),
                ("gpg", lambda r, m, u: ca.compute_gpg_outcome_advantage(token_level_rewards=r, response_mask=m, index=u))]
        if min(sizes) >= 2:
            for norm in (True, False):
                ests.append((f"grpo_passk_{'std' if norm else 'nostd'}",
                             lambda r, m, u, norm=norm: ca.compute_grpo_passk_outcome_advantage(
                                 token_level_rewards=r, response_mask=m, index=u,
                                 config=DictConfig(norm_adv_by_std_in_grpo=norm))))
        for est, fn in ests:
            adv, ret = fn(rewards.clone(), mask, uid)
            arrays.update({f"c{ci}_rewards": rewards, f"c{ci}_mask": mask, f"c{ci}_uid": np.array([str(u) for u in uid]),
                           f"c{ci}_adv": adv, f"c{ci}_ret": ret})
            cases.append({"name": name, "estimator": est})
            ci += 1
    for name, (B, R) in [("remax_a", (7, 12)), ("remax_b", (16, 33))]:
        rewards = torch.randn(B, R, generator=g) * (torch.rand(B, R, generator=g) > 0.6)
        mask = torch.ones(B, R, dtype=torch.int64)
        for i in range(B):
            mask[i, int(torch.randint(1, R + 1, (1,), generator=g)):] = 0
        base = torch.randn(B, generator=g)
        adv, ret = ca.compute_remax_outcome_advantage(token_level_rewards=rewards, reward_baselines=base,
                                                      response_mask=mask)
        arrays.update({f"c{ci}_rewards": rewards, f"c{ci}_mask": mask, f"c{ci}_baselines": base, f"c{ci}_adv": adv,
                       f"c{ci}_ret": ret})
        cases.append({"name": name, "estimator": "remax"})
        ci += 1
    # pass@k rejects singleton groups
    try:
        ca.compute_grpo_passk_outcome_advantage(token_level_rewards=torch.ones(3, 4), response_mask=torch.ones(3, 4),
                                                index=np.array(["a", "a", "b"], dtype=object),
                                                config=DictConfig(norm_adv_by_std_in_grpo=True))
        passk_error = ""
    except ValueError as e:
        passk_error = str(e)
    _save("more_adv.npz", arrays, {"cases": cases, "passk_singleton_error": passk_error,
                                   "ref": "core_algos.py:327-386, 495-546, 588-621, 624-684"})


def gen_rfpp():
    """REINFORCE++ (core_algos.py:550-586): masked discounted returns + masked_whiten."""
    g = torch.Generator().manual_seed(103)
    arrays, cases = {}, []
    for ci, (B, R, gamma, obs) in enumerate([(6, 20, 1.0, False), (8, 33, 0.99, True), (3, 9, 0.9, True)]):
        rewards = torch.randn(B, R, generator=g) * (torch.rand(B, R, generator=g) > 0.7)
        mask = torch.ones(B, R, dtype=torch.int64)
        for i in range(B):
            mask[i, int(torch.randint(2, R + 1, (1,), generator=g)):] = 0
        if obs:
            mask[:, 1] = 0  # observation tokens inside the response reset the carry
        adv, ret = ca.compute_reinforce_plus_plus_outcome_advantage(rewards, mask, config=DictConfig(gamma=gamma))
        arrays.update({f"c{ci}_rewards": rewards, f"c{ci}_mask": mask, f"c{ci}_adv": adv, f"c{ci}_ret": ret})
        cases.append({"gamma": gamma})
    _save("rfpp.npz", arrays, {"cases": cases, "ref": "core_algos.py:550-586"})


def gen_gpg_loss():
    """GPG policy loss (core_algos.py:957-975) composed as dp_actor.py:419-466 composes any registered loss."""
    g = torch.Generator().manual_seed(4321)
    arrays, cases = {}, []
    pg_fn = ca.get_policy_loss_fn("gpg")
    for ci, (shape, kind, mode, kl, ent_c, lsf) in enumerate([((6, 16), "edges", "token-mean", "low_var_kl", 0.001, 0.5),
                                                              ((8, 64), "random", "seq-mean-token-mean", "kl", 0.0, 1.0),
                                                              ((5, 33), "edges", "seq-mean-token-sum", "mse", 0.01, 0.25),
                                                              ((4, 40), "random", "seq-mean-token-sum-norm", "abs", 0.0, 1.0)]):
        old, logp, adv, mask, ent, ref = ppo_loss_inputs(g, *shape, kind)
        lp = logp.clone().requires_grad_(True)
        en = ent.clone().requires_grad_(True)
        pg_loss, c1, c2, c3 = pg_fn(old_log_prob=old, log_prob=lp, advantages=adv, response_mask=mask,
                                    loss_agg_mode=mode, config=None)
        entropy_loss = ca.agg_loss(loss_mat=en, loss_mask=mask, loss_agg_mode=mode)
        policy_loss = pg_loss - entropy_loss * ent_c if ent_c != 0 else pg_loss
        kld = ca.kl_penalty(logprob=lp, ref_logprob=ref, kl_penalty=kl)
        kl_loss = ca.agg_loss(loss_mat=kld, loss_mask=mask, loss_agg_mode=mode)
        loss = (policy_loss + kl_loss * 0.001) * lsf
        loss.backward()
        for k, v in dict(old_log_prob=old, log_prob=logp, advantages=adv, response_mask=mask, entropy=ent,
                         ref_log_prob=ref, out_pg_loss=pg_loss.detach(), out_loss=loss.detach(),
                         out_dlogp=lp.grad, out_dentropy=en.grad if en.grad is not None else torch.zeros_like(en),
                         out_clip=torch.tensor([float(c1), float(c2), float(c3)])).items():
            arrays[f"c{ci}_{k}"] = v
        cases.append(dict(loss_agg_mode=mode, kl_loss_type=kl, entropy_coeff=ent_c, kl_loss_coef=0.001,
                          loss_scale_factor=lsf, use_kl_loss=True))
    _save("gpg_loss.npz", arrays, {"cases": cases, "ref": "core_algos.py:957-975; dp_actor.py:419-466"})


def gen_seq_loss():
    """Sequence-level policy losses composed as dp_actor.py:419-466 composes any registered loss: GSPO
    (core_algos.py:892-954, sequence-mean log-ratio, seq-mean-token-mean pg aggregation) and GMPO geo_mean
    (:1143-1210, geometric-mean ratio of sign-clipped token log-ratios, mean over rows)."""
    from verl.workers.config import ActorConfig
    from verl.workers.config.optimizer import OptimizerConfig

    g = torch.Generator().manual_seed(5151)
    arrays, cases = {}, []
    specs = [("gspo", (6, 16), "edges", "token-mean", "low_var_kl", 0.001, 0.5, (0.2, 0.2)),
             ("gspo", (8, 40), "random", "seq-mean-token-sum", "kl", 0.0, 1.0, (0.2, 0.28)),
             ("gspo", (5, 33), "big", "seq-mean-token-mean", "abs", 0.01, 0.25, (0.0003, 0.0004)),
             ("geo_mean", (6, 16), "edges", "token-mean", "low_var_kl", 0.001, 0.5, (0.2, 0.2)),
             ("geo_mean", (8, 40), "random", "seq-mean-token-mean", "mse", 0.0, 1.0, (0.4, 0.4)),
             ("geo_mean", (5, 33), "big", "seq-mean-token-sum-norm", "kl", 0.01, 0.25, (0.05, 0.1))]
    for ci, (loss, shape, kind, mode, kl, ent_c, lsf, (clo, chi)) in enumerate(specs):
        old, logp, adv, mask, ent, ref = ppo_loss_inputs(g, *shape, "edges" if kind == "edges" else "random")
        if kind == "big":  # sequence log-ratios past GSPO's clamp at 10, every sign of advantage
            logp = logp + torch.randn(shape[0], 1, generator=g) * 12.0
            adv[1] = 0.0
        if loss == "geo_mean":  # GMPO uses a per-sequence advantage (outcome estimators): constant per row
            adv = adv[:, :1].expand_as(adv).clone()
        cfg = ActorConfig(strategy="fsdp", clip_ratio=0.2, clip_ratio_low=clo, clip_ratio_high=chi,
                          loss_agg_mode=mode, optim=OptimizerConfig(lr=1e-6), ppo_micro_batch_size_per_gpu=2,
                          ppo_mini_batch_size=4)
        pg_fn = ca.get_policy_loss_fn(loss)
        lp = logp.clone().requires_grad_(True)
        en = ent.clone().requires_grad_(True)
        pg_loss, c1, c2, c3 = pg_fn(old_log_prob=old, log_prob=lp, advantages=adv, response_mask=mask,
                                    loss_agg_mode=mode, config=cfg)
        entropy_loss = ca.agg_loss(loss_mat=en, loss_mask=mask, loss_agg_mode=mode)
        policy_loss = pg_loss - entropy_loss * ent_c if ent_c != 0 else pg_loss
        kld = ca.kl_penalty(logprob=lp, ref_logprob=ref, kl_penalty=kl)
        kl_loss = ca.agg_loss(loss_mat=kld, loss_mask=mask, loss_agg_mode=mode)
        loss_v = (policy_loss + kl_loss * 0.001) * lsf
        loss_v.backward()
        for k, v in dict(old_log_prob=old, log_prob=logp, advantages=adv, response_mask=mask, entropy=ent,
                         ref_log_prob=ref, out_pg_loss=pg_loss.detach(), out_loss=loss_v.detach(),
                         out_entropy_loss=entropy_loss.detach(), out_kl_loss=kl_loss.detach(),
                         out_dlogp=lp.grad, out_dentropy=en.grad if en.grad is not None else torch.zeros_like(en),
                         out_clip=torch.tensor([float(c1), float(c2), float(c3)])).items():
            arrays[f"c{ci}_{k}"] = v
        cases.append(dict(policy_loss=loss, loss_agg_mode=mode, kl_loss_type=kl, entropy_coeff=ent_c,
                          kl_loss_coef=0.001, loss_scale_factor=lsf, use_kl_loss=True, clip_ratio_low=clo,
                          clip_ratio_high=chi))
    _save("seq_loss.npz", arrays, {"cases": cases, "ref": "core_algos.py:892-954, 1143-1210; dp_actor.py:419-466"})


def gen_cov_loss():
    """Clip-Cov (core_algos.py:978-1069) and KL-Cov (:1072-1140) composed as dp_actor does. Clip-Cov's token subset
    comes from torch.randperm; these cases keep clip_num >= #candidates, where every candidate is taken and the
    result is deterministic (the subset draw itself is not reproducible outside torch's RNG)."""
    from verl.workers.config import ActorConfig
    from verl.workers.config.actor import PolicyLossConfig
    from verl.workers.config.optimizer import OptimizerConfig

    g = torch.Generator().manual_seed(6262)
    arrays, cases = {}, []
    specs = [("kl_cov", (6, 16), "token-mean", "low_var_kl", 0.001, 0.5, dict(kl_cov_ratio=0.05, ppo_kl_coef=0.1)),
             ("kl_cov", (8, 40), "seq-mean-token-mean", "kl", 0.0, 1.0, dict(kl_cov_ratio=0.0002, ppo_kl_coef=1.0)),
             ("kl_cov", (5, 33), "seq-mean-token-sum", "abs", 0.01, 0.25, dict(kl_cov_ratio=0.2, ppo_kl_coef=0.3)),
             ("clip_cov", (6, 16), "token-mean", "low_var_kl", 0.001, 0.5,
              dict(clip_cov_ratio=0.5, clip_cov_lb=1.0, clip_cov_ub=5.0)),
             ("clip_cov", (8, 40), "seq-mean-token-mean", "mse", 0.0, 1.0,
              dict(clip_cov_ratio=0.4, clip_cov_lb=0.5, clip_cov_ub=3.0)),
             ("clip_cov", (5, 33), "seq-mean-token-sum-norm", "kl", 0.01, 0.25,
              dict(clip_cov_ratio=0.9, clip_cov_lb=-1.0, clip_cov_ub=2.0))]
    for ci, (loss, shape, mode, kl, ent_c, lsf, pl) in enumerate(specs):
        old, logp, adv, mask, ent, ref = ppo_loss_inputs(g, *shape, "random")
        pcfg = PolicyLossConfig(loss_mode=loss, **pl)
        cfg = ActorConfig(strategy="fsdp", clip_ratio=0.2, clip_ratio_low=0.2, clip_ratio_high=0.28, loss_agg_mode=mode,
                          optim=OptimizerConfig(lr=1e-6), ppo_micro_batch_size_per_gpu=2, ppo_mini_batch_size=4,
                          policy_loss=pcfg)
        pg_fn = ca.get_policy_loss_fn(loss)
        lp = logp.clone().requires_grad_(True)
        en = ent.clone().requires_grad_(True)
        pg_loss, c1, c2, c3 = pg_fn(old_log_prob=old, log_prob=lp, advantages=adv, response_mask=mask,
                                    loss_agg_mode=mode, config=cfg)
        entropy_loss = ca.agg_loss(loss_mat=en, loss_mask=mask, loss_agg_mode=mode)
        policy_loss = pg_loss - entropy_loss * ent_c if ent_c != 0 else pg_loss
        kld = ca.kl_penalty(logprob=lp, ref_logprob=ref, kl_penalty=kl)
        kl_loss = ca.agg_loss(loss_mat=kld, loss_mask=mask, loss_agg_mode=mode)
        loss_v = (policy_loss + kl_loss * 0.001) * lsf
        loss_v.backward()
        for k, v in dict(old_log_prob=old, log_prob=logp, advantages=adv, response_mask=mask, entropy=ent,
                         ref_log_prob=ref, out_pg_loss=pg_loss.detach(), out_loss=loss_v.detach(),
                         out_dlogp=lp.grad, out_dentropy=en.grad if en.grad is not None else torch.zeros_like(en),
                         out_clip=torch.tensor([float(c1), float(c2), float(c3)])).items():
            arrays[f"c{ci}_{k}"] = v
        cases.append(dict(policy_loss=loss, loss_agg_mode=mode, kl_loss_type=kl, entropy_coeff=ent_c,
                          kl_loss_coef=0.001, loss_scale_factor=lsf, clip_ratio_low=0.2, clip_ratio_high=0.28,
                          cov_ratio=pl.get("clip_cov_ratio", pl.get("kl_cov_ratio")),
                          clip_cov_lb=pl.get("clip_cov_lb", 1.0), clip_cov_ub=pl.get("clip_cov_ub", 5.0),
                          ppo_kl_coef=pl.get("ppo_kl_coef", 0.1)))
    _save("cov_loss.npz", arrays, {"cases": cases, "ref": "core_algos.py:978-1140; dp_actor.py:419-466"})


# --------------------------------------------------------------------------------------------
# SURVEY §8(c) golden #7: the reference DataParallelPPOActor (dp_actor.py:300-482) on the tiny Qwen2, fp32:
# compute_log_prob (old log-probs + entropy) then update_policy over 2 mini-batches x 2 micro-batches with
# torch AdamW + clip_grad_norm_ (fsdp_workers.py:454-459, dp_actor.py:282-298). Records every actor/* metric
# list, the grad norms and the post-step parameters.
# --------------------------------------------------------------------------------------------
def _tiny_hf_causal():
    from safetensors.torch import load_file
    from transformers import Qwen2Config, Qwen2ForCausalLM

    cfg = Qwen2Config(**TINY_QWEN2, attn_implementation="eager")
    model = Qwen2ForCausalLM(cfg).float()
    sd = load_file(os.path.join(HERE, "tiny_qwen2", "model.safetensors"))
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert set(missing) <= {"lm_head.weight"} and not unexpected, (missing, unexpected)
    model.tie_weights()
    assert model.lm_head.weight.data_ptr() == model.model.embed_tokens.weight.data_ptr()
    return model


def _gloo_world1():
    import torch.distributed as dist

    if not dist.is_initialized():
        import socket

        s = socket.socket()
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
        s.close()
        dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)


def _ref_actor(model, cfgd, lr):
    """A reference DataParallelPPOActor in fp32: its torch.autocast(device_type=get_device_name()) is 'cpu' here,
    which would run the CPU bf16 autocast; the actor's device name is set to 'cuda' so autocast is disabled
    (no CUDA in this container) and the model runs in fp32 - the reference math without the bf16 casts."""
    import verl.workers.actor.dp_actor as ref_dp

    _gloo_world1()
    opt = torch.optim.AdamW(model.parameters(), lr=lr, betas=(0.9, 0.999), weight_decay=0.01) if lr else None
    actor = ref_dp.DataParallelPPOActor(DictConfig(cfgd), model, opt)
    actor.device_name = "cuda"
    return actor, opt


def _actor_cfg(**kw):
    d = dict(use_remove_padding=False, use_fused_kernels=False, ulysses_sequence_parallel_size=1,
             entropy_from_logits_with_chunking=False, use_torch_compile=False, entropy_checkpointing=False,
             ppo_mini_batch_size=4, ppo_micro_batch_size_per_gpu=2, ppo_epochs=1, use_dynamic_bsz=False,
             entropy_coeff=0.0, loss_agg_mode="token-mean", policy_loss=DictConfig(loss_mode="vanilla"),
             clip_ratio=0.2, clip_ratio_low=0.2, clip_ratio_high=0.2, clip_ratio_c=3.0, use_kl_loss=True,
             kl_loss_type="low_var_kl", kl_loss_coef=0.001, grad_clip=1.0)
    d.update(kw)
    return d


def _params(model):
    return {k: v.detach().clone() for k, v in model.state_dict().items() if k != "lm_head.weight"}


ACTOR_UPDATE_CASES = [
    # (name, actor config overrides, lr)
    ("grpo_k3", dict(), 1e-4),
    ("ent_seqmean_kl", dict(entropy_coeff=0.01, loss_agg_mode="seq-mean-token-mean", kl_loss_type="kl",
                            clip_ratio_high=0.28, clip_ratio_c=10.0), 1e-4),
]


def gen_actor_update():
    from verl import DataProto as RefDataProto

    z = np.load(os.path.join(HERE, "tiny_qwen2_rollout.npz"))
    seq, am, pos, resp = (torch.from_numpy(z[k]) for k in ("sequences", "attention_mask", "position_ids", "responses"))
    B, R = resp.shape
    B = 8  # 6 golden rows + 2 repeated rows with a shifted mask -> 2 mini-batches of 4 (2 micro-batches of 2)
    seq, am, pos, resp = (torch.cat([t, t[:2]], 0) for t in (seq, am, pos, resp))
    am[6, -3:] = 0  # shorter responses for the repeated rows
    am[7, -R + 1:] = 0
    g = torch.Generator().manual_seed(2024)
    arrays, cases = {}, []
    for ci, (name, over, lr) in enumerate(ACTOR_UPDATE_CASES):
        model = _tiny_hf_causal()
        before = _params(model)
        actor, opt = _ref_actor(model, _actor_cfg(**over), lr)
        data = RefDataProto.from_dict(tensors={"input_ids": seq, "attention_mask": am, "position_ids": pos,
                                               "responses": resp},
                                      meta_info={"micro_batch_size": 4, "temperature": 1.0, "use_dynamic_bsz": False})
        logp, ent = actor.compute_log_prob(data, calculate_entropy=True)
        rmask = am[:, -R:]
        old = (logp + 0.3 * torch.randn(B, R, generator=g)).detach()  # ratios across the clip bounds
        ref = (logp + 0.2 * torch.randn(B, R, generator=g)).detach()
        adv = torch.randn(B, 1, generator=g).expand(B, R) * rmask  # sequence-level advantages, +-
        adv = adv.contiguous()
        udata = RefDataProto.from_dict(tensors={"input_ids": seq, "attention_mask": am, "position_ids": pos,
                                                "responses": resp, "response_mask": rmask, "old_log_probs": old,
                                                "advantages": adv, "ref_log_prob": ref},
                                       meta_info={"temperature": 1.0})
        metrics = actor.update_policy(udata)
        after = _params(model)
        pre = f"c{ci}_"
        for k, v in dict(input_ids=seq, attention_mask=am, position_ids=pos, responses=resp, response_mask=rmask,
                         log_probs=logp, entropys=ent, old_log_probs=old, ref_log_prob=ref, advantages=adv).items():
            arrays[pre + k] = v
        for k, v in after.items():
            arrays[pre + "after." + k] = v
        cases.append(dict(name=name, config=_actor_cfg(**over), lr=lr, metrics=metrics,
                          param_sums={k: float(v.double().sum()) for k, v in after.items()},
                          delta_abs_sums={k: float((after[k] - before[k]).double().abs().sum()) for k in after}))
    for c in cases:
        c["config"]["policy_loss"] = dict(c["config"]["policy_loss"])
    _save("actor_update.npz", arrays, {"cases": cases, "weights": "tiny_qwen2/model.safetensors",
                                       "ref": "dp_actor.py:282-298, 300-359, 361-482; fsdp_workers.py:454-459",
                                       "precision": "fp32 (autocast disabled: actor.device_name='cuda' on a CPU box)"})


# --------------------------------------------------------------------------------------------
# One GRPO fit() step composed from the reference's own functions (ray_trainer.py:1104-1399) on the tiny
# Qwen2, fp32, greedy: HFRollout (hf_rollout.py:53-177) -> union -> compute_response_mask -> global_token_num
# -> reward (reward-model scores through NaiveRewardManager, naive.py:46-60; plus the gsm8k rule score of the
# same responses with a stub tokenizer, naive.py:62-122 + gsm8k.py) -> compute_log_prob (old + entropy ->
# actor/entropy) -> ref log-prob -> compute_advantage (GRPO) -> update_policy -> compute_data_metrics /
# compute_timing_metrics / compute_throughout_metrics (metric_utils.py) -> FlopsCounter MFU.
# --------------------------------------------------------------------------------------------
from stub_tokenizer import StubTokenizer  # noqa: E402  (shared with the tests)


GRPO_STEP_CASES = [
    # n = 2: real groups. Greedy copies of a prompt are identical, so the group-normalised advantages (+-1/sqrt 2)
    # cancel inside each micro-batch: the policy gradient is ~0 (the reference's too) and only the rollout,
    # reward, log-prob, advantage and metric composition is compared.
    dict(name="n2", n_prompts=4, n=2, P=12, R=10, pads=[0, 3, 0, 5], lr=1e-4, mini_prompts=2, micro=2,
         rm_scores=[1.0, 0.0, 0.5, 1.0, 0.0, 0.0, 1.0, 0.25], seed=99, compare_update=False),
    # n = 1: singleton groups (mean 0, std 1 -> A = score / (1 + 1e-6)): a real policy-gradient update
    dict(name="n1", n_prompts=8, n=1, P=12, R=10, pads=[0, 3, 0, 5, 1, 0, 2, 0], lr=1e-4, mini_prompts=4, micro=2,
         rm_scores=[1.0, 0.0, 0.5, 1.0, 0.0, -0.5, 1.0, 0.25], seed=7, compare_update=True),
    # groups of 2 DISTINCT responses (uid pairs over 8 different prompts, n = 1): the group-normalised advantages
    # (+-1/sqrt 2 by score order, 0 for a tie) do not cancel, so the post-update parameters are compared too
    dict(name="pairs", n_prompts=8, n=1, P=12, R=10, pads=[2, 0, 0, 4, 0, 1, 3, 0], lr=1e-4, mini_prompts=4, micro=2,
         rm_scores=[1.0, 0.0, 0.25, 0.75, 0.5, 0.5, -1.0, 1.0], seed=23, compare_update=True, uid_pairs=True),
]
GRPO_TIMING = {"gen": 0.5, "reward": 0.01, "old_log_prob": 0.2, "ref": 0.2, "adv": 0.01, "update_actor": 0.8,
               "step": 1.75}


def gen_grpo_step():
    arrays, metas = {}, []
    for ci, S in enumerate(GRPO_STEP_CASES):
        a, m = _grpo_step_case(S)
        arrays.update({f"c{ci}_{k}": v for k, v in a.items()})
        metas.append(m)
    _save("grpo_step.npz", arrays, {"cases": metas})


def _grpo_step_case(S):
    import verl.trainer.ppo.ray_trainer as rt
    import verl.workers.rollout.hf_rollout as ref_hf
    from verl import DataProto as RefDataProto
    from verl.trainer.ppo.metric_utils import (compute_data_metrics, compute_throughout_metrics,
                                               compute_timing_metrics)
    from verl.utils.flops_counter import FlopsCounter
    from verl.workers.reward_manager.naive import NaiveRewardManager

    model = _tiny_hf_causal()
    before = _params(model)
    g = torch.Generator().manual_seed(S["seed"])
    Np, P, R, n = S["n_prompts"], S["P"], S["R"], S["n"]
    ids = torch.randint(3, 512, (Np, P), generator=g)
    am = torch.ones(Np, P, dtype=torch.int64)
    for i, npad in enumerate(S["pads"]):
        am[i, :npad] = 0
        ids[i, :npad] = TINY_QWEN2["pad_token_id"]
    pos = compute_position_id_with_mask(am)

    ref_hf.get_device_name = lambda: "cuda"  # fp32 generate (autocast disabled on this CPU box)
    if not hasattr(torch.cpu, "empty_cache"):  # hf_rollout.py:174 calls the device's empty_cache (a no-op here)
        torch.cpu.empty_cache = lambda: None
    rollout = ref_hf.HFRollout(model, DictConfig(do_sample=False, temperature=1.0, response_length=R, top_p=1.0,
                                                 top_k=-1, val_kwargs=DictConfig()))

    def run_rollout(eos):
        batch = RefDataProto.from_single_dict({"input_ids": ids, "attention_mask": am, "position_ids": pos,
                                               "data_source": np.array(["openai/gsm8k"] * Np, dtype=object),
                                               "reward_model": np.array([{"ground_truth": None} for _ in range(Np)],
                                                                        dtype=object)})
        batch.non_tensor_batch["uid"] = np.array([f"uid{i}" for i in range(Np)], dtype=object)
        gen_batch = batch.pop(batch_keys=["input_ids", "attention_mask", "position_ids"])
        gen_batch.meta_info.update({"eos_token_id": eos, "pad_token_id": TINY_QWEN2["pad_token_id"]})
        gen_batch = gen_batch.repeat(repeat_times=n, interleave=True)
        out = rollout.generate_sequences(gen_batch)
        batch = batch.repeat(repeat_times=n, interleave=True)
        return batch.union(out)

    batch = run_rollout(TINY_QWEN2["eos_token_id"])
    eos = int(batch.batch["responses"][2 if n > 1 else 1, 3])  # some rows stop mid-response
    batch = run_rollout(eos)
    if S.get("uid_pairs"):  # rows (2i, 2i + 1) form one GRPO group
        batch.non_tensor_batch["uid"] = np.array([f"pair{i // 2}" for i in range(Np * n)], dtype=object)
    B = Np * n
    batch.batch["response_mask"] = rt.compute_response_mask(batch)
    batch.meta_info["global_token_num"] = torch.sum(batch.batch["attention_mask"], dim=-1).tolist()

    # rule reward (gsm8k strict) on the same responses: ground truth = the extracted answer for even prompts,
    # a different digit for odd ones
    from verl.utils.reward_score import gsm8k

    tok = StubTokenizer()
    gts = []
    for i in range(Np):
        r = batch.batch["responses"][i * n]
        vl = int(batch.batch["attention_mask"][i * n, P:].sum())
        ans = gsm8k.extract_solution(tok.decode(r[:vl]), "strict")
        gts.append(str(ans) if (i % 2 == 0 and ans is not None) else "9")
    for i in range(B):
        batch.non_tensor_batch["reward_model"][i] = {"ground_truth": gts[i // n]}
    rule = NaiveRewardManager(tokenizer=tok, num_examine=0)(batch, return_dict=True)
    rule_scores = rule["reward_tensor"]

    # reward-model scores (preset per row) placed at the last valid response token; the naive manager returns
    # rm_scores as the reward tensor (naive.py:55-60)
    vl = batch.batch["attention_mask"][:, P:].sum(-1)
    rm = torch.zeros(B, R)
    rm[torch.arange(B), vl - 1] = torch.tensor(S["rm_scores"])
    batch.batch["rm_scores"] = rm
    reward_tensor = NaiveRewardManager(tokenizer=tok, num_examine=0)(batch, return_dict=True)["reward_tensor"]

    mini = S["mini_prompts"] * n  # fsdp_workers.py:209-214 normalisation at dp=1
    actor, opt = _ref_actor(model, _actor_cfg(ppo_mini_batch_size=mini, ppo_micro_batch_size_per_gpu=S["micro"]),
                            S["lr"])
    batch.meta_info["micro_batch_size"] = 4
    batch.meta_info["temperature"] = 1.0
    batch.meta_info["use_dynamic_bsz"] = False
    old, ent = actor.compute_log_prob(batch, calculate_entropy=True)
    actor_entropy = ca.agg_loss(loss_mat=ent, loss_mask=batch.batch["response_mask"], loss_agg_mode="token-mean")
    ref_model = _tiny_hf_causal()
    ref_actor, _ = _ref_actor(ref_model, _actor_cfg(), None)
    ref_lp, _ = ref_actor.compute_log_prob(batch, calculate_entropy=False)
    batch.batch["old_log_probs"] = old
    batch.batch["ref_log_prob"] = ref_lp
    batch.batch["token_level_scores"] = reward_tensor
    batch.batch["token_level_rewards"] = batch.batch["token_level_scores"]
    batch = rt.compute_advantage(batch, adv_estimator="grpo", norm_adv_by_std_in_grpo=True, num_repeat=n)
    batch.meta_info.pop("micro_batch_size")
    metrics = actor.update_policy(batch)
    after = _params(model)
    timing = dict(GRPO_TIMING)
    dm = compute_data_metrics(batch, use_critic=False)
    tm = compute_timing_metrics(batch, timing)
    th = compute_throughout_metrics(batch, timing, n_gpus=1)
    from transformers import Qwen2Config

    fc = FlopsCounter(Qwen2Config(**TINY_QWEN2))
    est, _ = fc.estimate_flops(batch.meta_info["global_token_num"], timing["update_actor"])
    big = FlopsCounter(Qwen2Config(vocab_size=151936, hidden_size=896, intermediate_size=4864, num_hidden_layers=24,
                                   num_attention_heads=14, num_key_value_heads=2))
    est_big, _ = big.estimate_flops([768] * 512, 1.0)
    arrays = dict(prompt_ids=ids, prompt_attention_mask=am, prompt_position_ids=pos, rm_scores_preset=torch.tensor(
        S["rm_scores"]), rule_scores=rule_scores, token_level_scores=reward_tensor)
    for k in ("prompts", "responses", "input_ids", "attention_mask", "position_ids", "response_mask",
              "old_log_probs", "ref_log_prob", "advantages", "returns"):
        arrays[k] = batch.batch[k]
    arrays["entropys"] = ent
    for k, v in after.items():
        arrays["after." + k] = v
    meta = dict(S, eos_token_id=eos, pad_token_id=TINY_QWEN2["pad_token_id"], ground_truths=gts,
                uid_groups=[i // n for i in range(B)], actor_entropy=float(actor_entropy), update_metrics=metrics,
                data_metrics={k: float(v) for k, v in dm.items()}, timing_metrics={k: float(v) for k, v in tm.items()},
                throughput_metrics={k: float(v) for k, v in th.items()}, flops_tiny_tflops=float(est),
                flops_qwen05b_768x512_tflops=float(est_big),
                param_sums={k: float(v.double().sum()) for k, v in after.items()},
                delta_abs_sums={k: float((after[k] - before[k]).double().abs().sum()) for k in after},
                actor_config=dict(_actor_cfg(ppo_mini_batch_size=mini, ppo_micro_batch_size_per_gpu=S["micro"]),
                                  policy_loss={"loss_mode": "vanilla"}),
                ref="ray_trainer.py:196-291,1104-1399; hf_rollout.py:53-177; naive.py:46-122; gsm8k.py:52; "
                    "dp_actor.py:300-482; metric_utils.py:80-302; flops_counter.py:135-167",
                precision="fp32 (autocast disabled)")
    return arrays, meta


# --------------------------------------------------------------------------------------------
# Config #2 at full depth: the reference HF Qwen2ForCausalLM (what the FSDP/HF path loads for Qwen2.5-0.5B)
# on deterministic CPU-seeded weights (tests/golden/full_depth.py; never committed), fp32: greedy generate of
# 4 x 64-token prompts for 64 tokens post-processed as HFRollout (hf_rollout.py:112-171) with the top-2 logit
# margin of every step, teacher-forced log-probs / entropy as dp_actor.py:249-272 computes them, and the size
# of the CPU bf16-autocast logit error on the same sequences (the bf16 margin bound the test uses).
# --------------------------------------------------------------------------------------------
def gen_full_depth():
    import full_depth as fd
    from transformers import Qwen2Config, Qwen2ForCausalLM

    cfg = Qwen2Config(**fd.QWEN25_05B, attn_implementation="eager")
    model = Qwen2ForCausalLM(cfg).float()  # built on the CPU (a meta-device build leaves RoPE's inv_freq unset)
    sd = fd.make_state_dict()
    missing, unexpected = model.load_state_dict(sd, strict=False)
    assert set(missing) == {"lm_head.weight"} and not unexpected
    model.tie_weights()
    model.eval()
    ids, am, pos = fd.prompts()
    B, P = ids.shape
    R = 64
    eos, pad = fd.QWEN25_05B["eos_token_id"], fd.QWEN25_05B["pad_token_id"]
    with torch.no_grad():
        out = model.generate(input_ids=ids, attention_mask=am, position_ids=pos, do_sample=False, num_beams=1,
                             max_new_tokens=R, eos_token_id=eos, pad_token_id=pad, output_scores=True,
                             return_dict_in_generate=True, use_cache=True)
    seq = out.sequences
    if seq.shape[1] < P + R:
        seq = torch.cat([seq, torch.full((B, P + R - seq.shape[1]), pad)], 1)
    top2 = torch.stack([torch.topk(s, 2, -1).values for s in out.scores], 1)  # (B, steps, 2)
    gaps = torch.full((B, R), float("inf"))
    gaps[:, :top2.shape[1]] = top2[..., 0] - top2[..., 1]
    resp = seq[:, P:]
    rmask = vF.get_response_mask(resp, eos_token=eos, dtype=am.dtype)
    full_am = torch.cat([am, rmask], -1)
    full_pos = torch.cat([pos, pos[:, -1:] + torch.arange(1, R + 1).unsqueeze(0)], -1)
    with torch.no_grad():
        logits = model(input_ids=seq, attention_mask=full_am, position_ids=full_pos, use_cache=False).logits
        lg = logits[:, -R - 1:-1]
        logp = vF.logprobs_from_logits_v2(lg, resp)
        ent = vF.entropy_from_logits(lg)
        with torch.autocast("cpu", dtype=torch.bfloat16):
            lb = model(input_ids=seq, attention_mask=full_am, position_ids=full_pos, use_cache=False).logits
        lbr = lb.float()[:, -R - 1:-1]
        err = (lbr - lg).abs()
        err_max_row = err.amax(-1)  # (B, R): worst logit error of the bf16 model at each response step
        t2 = torch.topk(lg, 2, -1).indices  # the fp32 reference's top-2 tokens of each teacher-forced step
        d32 = lg.gather(-1, t2[..., :1]) - lg.gather(-1, t2[..., 1:])
        d16 = lbr.gather(-1, t2[..., :1]) - lbr.gather(-1, t2[..., 1:])
        gap_err = (d16 - d32).abs().squeeze(-1)  # (B, R): bf16 error of the top-2 margin itself
        logp_bf16 = vF.logprobs_from_logits_v2(lb.float()[:, -R - 1:-1], resp)
        # the teacher-forced reference logits of every response step, summarised (the full (4, 64, V) block is
        # 155 MB): the 32 largest with their token ids, the logsumexp, and the CPU bf16 model's values at those ids
        topv, topi = torch.topk(lg, 32, -1)
        lse = torch.logsumexp(lg.double(), -1).float()
        bf_at_top = lbr.gather(-1, topi)
    arrays = dict(prompt_ids=ids, prompt_attention_mask=am, prompt_position_ids=pos, sequences=seq, responses=resp,
                  attention_mask=full_am, position_ids=full_pos, top2_gap=gaps, log_probs=logp, entropy=ent,
                  cpu_bf16_logit_err=err_max_row, cpu_bf16_gap_err=gap_err, cpu_bf16_log_probs=logp_bf16,
                  ref_top32_ids=topi, ref_top32_logits=topv, ref_lse=lse, cpu_bf16_top32_logits=bf_at_top)
    _save("full_depth.npz", arrays, {
        "eos_token_id": eos, "pad_token_id": pad, "response_length": R, "weights": "full_depth.make_state_dict()",
        "scales": fd.SCALES, "seed": fd.SEED, "weight_checksum": fd.checksum(sd), "min_top2_gap": float(gaps.min()),
        "median_top2_gap": float(gaps[torch.isfinite(gaps)].median()),
        "cpu_bf16_logit_err_max": float(err_max_row.max()), "cpu_bf16_logit_err_median": float(err_max_row.median()),
        "cpu_bf16_logp_err_max": float((logp_bf16 - logp).abs().max()),
        "cpu_bf16_gap_err_max": float(gap_err.max()), "cpu_bf16_gap_err_median": float(gap_err.median()),
        "hf": "transformers Qwen2ForCausalLM fp32 eager attention", "ref": "hf_rollout.py:112-171; dp_actor.py:249-272"})


# --------------------------------------------------------------------------------------------
# Configs #4 / #5 at full width, 2 decoder layers (tests/golden/wide.py weights, never committed), fp32 on the CPU:
# config #4 (Llama-3-8B): actor log-probs / entropy (dp_actor.py:249-272), the vanilla PPO loss's backward (per-tensor
# gradient norms), the critic (LlamaForTokenClassification, num_labels 1: dp_critic.py:127-145 values slice), its
# value-loss backward (dp_critic.py:218-245) and GAE over its values (core_algos.py:208-256); config #5 (Qwen2.5-7B):
# actor log-probs / entropy / loss backward. The CPU bf16-autocast model's log-probs and values size the bf16 bound.
# --------------------------------------------------------------------------------------------
def gen_wide():
    import wide
    from transformers import LlamaConfig, LlamaForCausalLM, LlamaForTokenClassification, Qwen2Config, Qwen2ForCausalLM

    arrays, meta = {}, {}
    for which in ("llama", "qwen7b"):
        cfgd = wide.LLAMA3_8B_W if which == "llama" else wide.QWEN25_7B_W
        sd = wide.make_state_dict(which)
        ids, am, pos, R = wide.sequences(which)
        resp = ids[:, -R:]
        rmask = am[:, -R:]
        if which == "llama":
            cfg = LlamaConfig(**cfgd, attn_implementation="eager", mlp_bias=False)
            actor = LlamaForCausalLM(cfg).float()
        else:
            cfg = Qwen2Config(**cfgd, attn_implementation="eager")
            actor = Qwen2ForCausalLM(cfg).float()
        missing, unexpected = actor.load_state_dict({k: v for k, v in sd.items() if not k.startswith("score")},
                                                    strict=True), None
        g = torch.Generator().manual_seed(4 if which == "llama" else 5)
        lg = actor(input_ids=ids, attention_mask=am, position_ids=pos, use_cache=False).logits[:, -R - 1:-1]
        logp = vF.logprobs_from_logits_v2(lg, resp)
        ent = vF.entropy_from_logits(lg)
        old = logp.detach() + 0.05 * torch.randn(logp.shape, generator=g)
        adv = torch.randn(logp.shape, generator=g)
        pg, _, _, _ = ca.compute_policy_loss_vanilla(old_log_prob=old, log_prob=logp, advantages=adv,
                                                     response_mask=rmask, loss_agg_mode="token-mean",
                                                     config=DictConfig(_actor_cfg()))
        pg.backward()
        gnorm = {k: float(p.grad.double().norm()) for k, p in actor.named_parameters()}
        with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
            lb = actor(input_ids=ids, attention_mask=am, position_ids=pos, use_cache=False).logits
        logp_bf16 = vF.logprobs_from_logits_v2(lb.float()[:, -R - 1:-1], resp)
        p = f"{which}_"
        arrays.update({p + "input_ids": ids, p + "attention_mask": am, p + "position_ids": pos, p + "log_probs": logp,
                       p + "entropy": ent, p + "old_log_probs": old, p + "advantages": adv, p + "pg_loss": pg.detach(),
                       p + "cpu_bf16_log_probs": logp_bf16})
        meta[which] = {"grad_norms": gnorm, "response_length": R, "weight_checksum": wide.checksum(sd),
                       "cpu_bf16_logp_err_max": float((logp_bf16 - logp).abs().max())}
        del actor, lg, lb
        if which == "llama":
            cfgc = LlamaConfig(**cfgd, attn_implementation="eager", mlp_bias=False, num_labels=1,
                               classifier_dropout=0.0)
            critic = LlamaForTokenClassification(cfgc).float()
            csd = {k: v for k, v in sd.items() if not k.startswith("lm_head")}
            critic.load_state_dict(csd, strict=True)
            critic.train()
            vpreds = critic(input_ids=ids, attention_mask=am, position_ids=pos, use_cache=False).logits
            vpreds = vpreds[:, -R - 1:-1].squeeze(-1)
            with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
                vb = critic(input_ids=ids, attention_mask=am, position_ids=pos, use_cache=False).logits
            vb = vb.float()[:, -R - 1:-1].squeeze(-1)
            # token-level rewards: a score at the last valid response token (GAE over the critic's own values)
            scores = torch.tensor([1.0, -0.5])
            vl = rmask.sum(-1)
            rewards = torch.zeros(ids.shape[0], R)
            rewards[torch.arange(ids.shape[0]), vl - 1] = scores
            adv_g, ret_g = ca.compute_gae_advantage_return(rewards, vpreds.detach(), rmask, gamma=1.0, lam=0.95)
            values_old = (vpreds.detach() + 0.1 * torch.randn(vpreds.shape, generator=g)) * rmask
            vf_loss, vf_clipfrac = ca.compute_value_loss(vpreds=vpreds, returns=ret_g, values=values_old,
                                                         response_mask=rmask, cliprange_value=0.5,
                                                         loss_agg_mode="token-mean")
            (vf_loss * 0.5).backward()
            cnorm = {k: float(q.grad.double().norm()) for k, q in critic.named_parameters()}
            arrays.update({p + "values": vpreds.detach(), p + "cpu_bf16_values": vb, p + "token_level_rewards": rewards,
                           p + "gae_advantages": adv_g, p + "gae_returns": ret_g, p + "values_old": values_old,
                           p + "vf_loss": vf_loss.detach(), p + "vf_clipfrac": vf_clipfrac})
            meta[which].update(critic_grad_norms=cnorm, gamma=1.0, lam=0.95, cliprange_value=0.5,
                               cpu_bf16_value_err_max=float((vb - vpreds.detach()).abs().max()))
            del critic
        del sd
    meta["ref"] = ("dp_actor.py:249-272, core_algos.py:815-889 (vanilla, token-mean), dp_critic.py:127-145, 218-245, "
                   "core_algos.py:208-256, 1230-1269; HF LlamaForCausalLM / LlamaForTokenClassification / "
                   "Qwen2ForCausalLM fp32 eager attention")
    _save("wide.npz", arrays, meta)


# --------------------------------------------------------------------------------------------
# LR schedules (fsdp_workers.py:461-486): the reference's LambdaLR over a real torch optimizer, the lr read with
# get_last_lr() before each lr_scheduler.step() as update_actor does (fsdp_workers.py:717-719)
# --------------------------------------------------------------------------------------------
def gen_lr_schedule():
    cases = [dict(warmup_style="constant", lr_warmup_steps=-1, lr_warmup_steps_ratio=0.0, total_training_steps=20),
             dict(warmup_style="constant", lr_warmup_steps=5, total_training_steps=20),
             dict(warmup_style="constant", lr_warmup_steps=-1, lr_warmup_steps_ratio=0.25, total_training_steps=20),
             dict(warmup_style="cosine", lr_warmup_steps=-1, lr_warmup_steps_ratio=0.0, total_training_steps=20),
             dict(warmup_style="cosine", lr_warmup_steps=4, total_training_steps=30, min_lr_ratio=0.1),
             dict(warmup_style="cosine", lr_warmup_steps=3, total_training_steps=25, min_lr_ratio=0.0, num_cycles=1.5),
             dict(warmup_style="cosine", lr_warmup_steps=-1, lr_warmup_steps_ratio=0.1, total_training_steps=40,
                  min_lr_ratio=0.05, num_cycles=0.5)]
    lrs = []
    for c in cases:
        total = c.get("total_training_steps", 0)
        warm = int(c.get("lr_warmup_steps", -1))
        if warm < 0:
            warm = int(c.get("lr_warmup_steps_ratio", 0.0) * total)
        opt = torch.optim.AdamW([torch.nn.Parameter(torch.zeros(1))], lr=1e-6)
        if c["warmup_style"] == "constant":
            sch = vF.get_constant_schedule_with_warmup(optimizer=opt, num_warmup_steps=warm)
        else:
            sch = vF.get_cosine_schedule_with_warmup(optimizer=opt, num_warmup_steps=warm, num_training_steps=total,
                                                     min_lr_ratio=c.get("min_lr_ratio", 0.0),
                                                     num_cycles=c.get("num_cycles", 0.5))
        seq = []
        for _ in range(total + 5):
            seq.append(sch.get_last_lr()[0])
            opt.step()
            sch.step()
        lrs.append(seq)
    width = max(len(s) for s in lrs)
    arr = np.full((len(cases), width), np.nan)
    for i, s in enumerate(lrs):
        arr[i, :len(s)] = s
    _save("lr_schedule.npz", dict(lr=arr), {"cases": cases, "base_lr": 1e-6,
                                            "ref": "fsdp_workers.py:461-486, torch_functional.py:509-575"})


def gen_bf16_update(grouped=False):
    """The reference DataParallelPPOActor (dp_actor.py:300-482) at Qwen2.5-0.5B width (4 layers, full vocabulary,
    tied lm_head; tests/golden/bf16_update.py) run twice on the same inputs: in fp32 (autocast disabled, as
    _ref_actor) and under its own torch.autocast(bf16) (dp_actor.py:110; on this CPU box the device name is 'cpu',
    so the CPU bf16 autocast runs). SDPA attention (fp32 score accumulation like the GPU's flash-attn). Recorded for
    both runs: log-probs / entropy, every update metric, per-tensor gradient norms and a fixed sample of gradient
    elements (captured when _optimizer_step calls clip_grad_norm_: the accumulated gradient of the 2 micro-batches,
    before clipping),
    and the same sample of the parameter update. The bf16-vs-fp32 difference of the reference itself is the
    yardstick the production bf16 path is held to (tests/test_bf16_update_gpu.py).

    ``grouped``: the same on bf16_update.batch(grouped=True) — 4 prompts x n = 4 in the trainer's interleaved repeat
    — so the GPU side runs prefix sharing (qwen2.PrefixShare, flash q_start, drl_sum_rows) under the same bar; the
    reference itself runs every row in full (it has no prefix sharing) -> bf16_update_grouped.npz."""
    import bf16_update as bu
    import verl.workers.actor.dp_actor as ref_dp
    from transformers import Qwen2Config, Qwen2ForCausalLM
    from verl import DataProto as RefDataProto

    # the GPU reference computes log-probs with flash-attn's cross-entropy (torch_functional.py:81-88: fp32 math over
    # the bf16 logits, fp32 result); this CPU box has no flash-attn, and the torch fallback (logprobs_from_logits_v2)
    # would run log_softmax in bf16 and return bf16 log-probs. The fp32-math fallback stands in for flash-attn here.
    ref_dp.logprobs_from_logits = lambda logits, labels, inplace_backward=True: vF.logprobs_from_logits_v2(
        logits.float(), labels)
    sd = bu.make_state_dict()
    bt = bu.batch(grouped)
    lr = 1e-5
    acfg = _actor_cfg(entropy_coeff=0.001, ppo_mini_batch_size=bu.B, ppo_micro_batch_size_per_gpu=bu.B // 2)
    arrays = {k: v for k, v in bt.items() if not k.startswith("noise")}
    meta = {"config": dict(acfg, policy_loss=dict(acfg["policy_loss"])), "lr": lr, "model": bu.CFG,
            "weight_checksum": bu.checksum(sd), "runs": {}, "grouped": bool(grouped)}
    old = ref = None
    embed_idx = bu.embed_rows_index(bt["input_ids"].numpy())
    for mode in ("fp32", "bf16"):
        torch.manual_seed(0)
        model = Qwen2ForCausalLM(Qwen2Config(**bu.CFG, attn_implementation="sdpa")).float()
        missing, unexpected = model.load_state_dict(sd, strict=False)
        assert set(missing) <= {"lm_head.weight"} and not unexpected, (missing, unexpected)
        model.tie_weights()
        actor, opt = _ref_actor(model, acfg, lr)
        actor.device_name = "cuda" if mode == "fp32" else "cpu"  # "cpu": the reference's autocast(bf16) on CPU
        grads = {}
        clip0 = torch.nn.utils.clip_grad_norm_

        def clip(params, *a, _g=grads, _m=model, _c=clip0, **k):  # the gradient as accumulated, before clipping
            for n, prm in _m.named_parameters():
                _g[n] = prm.grad.detach().clone()
            return _c(params, *a, **k)

        torch.nn.utils.clip_grad_norm_ = clip
        data = RefDataProto.from_dict(tensors={k: bt[k] for k in ("input_ids", "attention_mask", "position_ids",
                                                                   "responses")},
                                      meta_info={"micro_batch_size": bu.B // 2, "temperature": 1.0,
                                                 "use_dynamic_bsz": False})
        logp, ent = actor.compute_log_prob(data, calculate_entropy=True)
        assert torch.isfinite(logp).all() and torch.isfinite(ent).all()
        if mode == "fp32":
            rm = bt["response_mask"]
            old = ((logp + 0.3 * bt["noise_old"]) * rm).detach()
            ref = ((logp + 0.2 * bt["noise_ref"]) * rm).detach()
        before = {n: q.detach().clone() for n, q in model.named_parameters()}
        udata = RefDataProto.from_dict(tensors={**{k: bt[k] for k in ("input_ids", "attention_mask", "position_ids",
                                                                      "responses", "response_mask", "advantages")},
                                                "old_log_probs": old, "ref_log_prob": ref},
                                       meta_info={"temperature": 1.0})
        metrics = actor.update_policy(udata)
        torch.nn.utils.clip_grad_norm_ = clip0
        assert len(grads) > 0
        run = {"metrics": {k: [float(x) for x in v] for k, v in metrics.items()},
               "grad_norms": {n: float(g.double().norm()) for n, g in grads.items()},
               "delta_abs_sums": {n: float((q.detach() - before[n]).double().abs().sum())
                                  for n, q in model.named_parameters()}}
        meta["runs"][mode] = run
        arrays[f"{mode}_log_probs"] = logp.detach().float()
        arrays[f"{mode}_entropys"] = ent.detach().float()  # bf16 in the autocast run (entropy_from_logits on bf16)
        for n, g in grads.items():
            idx = embed_idx if n == "model.embed_tokens.weight" else bu.sample_index(n, g.numel())
            arrays[f"{mode}_grad.{n}"] = g.reshape(-1)[torch.from_numpy(idx)]
            arrays[f"{mode}_delta.{n}"] = (dict(model.named_parameters())[n].detach() - before[n]).reshape(-1)[
                torch.from_numpy(idx)]
        del model, actor, opt, grads
    arrays["old_log_probs"], arrays["ref_log_prob"] = old, ref
    meta["ref"] = ("dp_actor.py:110 (autocast bf16), 300-482 (compute_log_prob, update_policy), 282-298 (clip + step); "
                   "fsdp_workers.py:454-459 (AdamW); HF Qwen2ForCausalLM, SDPA attention")
    _save("bf16_update_grouped.npz" if grouped else "bf16_update.npz", arrays, meta)


def gen_bf16_update_grouped():
    gen_bf16_update(grouped=True)


def gen_deep():
    """Configs #4 / #5 at FULL depth (tests/golden/deep.py: Llama-3-8B 32 layers, Qwen2.5-7B 28 layers, counter-hash
    weights): the reference HF models in fp32 (SDPA attention) and under the CPU bf16 autocast on 2 x (32 + 32)
    tokens, teacher-forced: the response tokens' log-probs, entropy, logsumexp and the top-32 logits of every
    response-predicting position (the bf16 run at the fp32 run's top-32 ids). Built on the meta device and filled
    tensor by tensor, so one 30 GB model is in memory at a time."""
    import deep
    from transformers import LlamaConfig, LlamaForCausalLM, Qwen2Config, Qwen2ForCausalLM
    from transformers.models.llama.modeling_llama import LlamaRotaryEmbedding
    from transformers.models.qwen2.modeling_qwen2 import Qwen2RotaryEmbedding

    arrays, meta = {}, {"ref": "HF LlamaForCausalLM / Qwen2ForCausalLM as fsdp_workers.py:244-330 loads them; "
                               "logits -> log_softmax / entropy as dp_actor.py:263-272", "models": {}}
    for which in ("llama", "qwen7b"):
        cfgd = deep.MODELS[which]
        if which == "llama":
            cfg = LlamaConfig(**{k: v for k, v in cfgd.items() if k != "attention_bias"}, attention_bias=False,
                              mlp_bias=False, attn_implementation="sdpa")
            with torch.device("meta"):
                model = LlamaForCausalLM(cfg)
        else:
            cfg = Qwen2Config(**cfgd, attn_implementation="sdpa")
            with torch.device("meta"):
                model = Qwen2ForCausalLM(cfg)
        model = model.to_empty(device="cpu")
        params = dict(model.named_parameters())
        digest_sd = {}
        for t, (name, shape) in enumerate(deep.hf_shapes(which)):
            x = deep.tensor_np(which, t, name, shape)
            with torch.no_grad():
                params[name].copy_(x)
            v = x.reshape(-1)
            digest_sd[name] = v[torch.linspace(0, v.numel() - 1, 4096, dtype=torch.float64).long()].clone()
            del x
        assert set(params) == {n for n, _ in deep.hf_shapes(which)}, set(params) ^ {n for n, _ in deep.hf_shapes(which)}
        model.model.rotary_emb = (LlamaRotaryEmbedding if which == "llama" else Qwen2RotaryEmbedding)(config=cfg)
        model.eval()
        ids, am, pos = deep.sequences(which)
        P, R = deep.P, deep.R
        resp = ids[:, P:]
        with torch.no_grad():
            lg = model(input_ids=ids, attention_mask=am, position_ids=pos, use_cache=False).logits[:, P - 1:P + R - 1]
            lg = lg.float()
            lsm = torch.log_softmax(lg, -1)
            lp = lsm.gather(-1, resp.unsqueeze(-1)).squeeze(-1)
            ent = -(lsm.exp() * lsm).sum(-1)
            lse = torch.logsumexp(lg, -1)
            top_l, top_i = lg.topk(32, -1)
            with torch.autocast("cpu", dtype=torch.bfloat16):
                lb = model(input_ids=ids, attention_mask=am, position_ids=pos, use_cache=False).logits[:, P - 1:P + R - 1]
            lb = lb.float()
            lsb = torch.log_softmax(lb, -1)
        p = f"{which}_"
        arrays.update({p + "input_ids": ids, p + "attention_mask": am, p + "position_ids": pos, p + "log_probs": lp,
                       p + "entropy": ent, p + "lse": lse, p + "top32_ids": top_i, p + "top32_logits": top_l,
                       p + "cpu_bf16_log_probs": lsb.gather(-1, resp.unsqueeze(-1)).squeeze(-1),
                       p + "cpu_bf16_top32_logits": lb.gather(-1, top_i), p + "cpu_bf16_lse": torch.logsumexp(lb, -1),
                       p + "cpu_bf16_entropy": -(lsb.exp() * lsb).sum(-1)})
        meta["models"][which] = {"config": cfgd, "weight_digest": deep.sample_digest(digest_sd), "P": P, "R": R,
                                 "cpu_bf16_logp_err_max": float((arrays[p + "cpu_bf16_log_probs"] - lp).abs().max())}
        print(which, meta["models"][which]["cpu_bf16_logp_err_max"], flush=True)
        del model, params, lg, lb, lsm, lsb
    _save("deep.npz", arrays, meta)


def gen_debug_metrics():
    """utils/debug/metrics.py:63-108 calculate_debug_metrics (ray_trainer.py:1221-1225) on seeded rollout / actor
    log-probs: with a response_mask, and with only an attention_mask (prompt + response columns)."""
    from types import SimpleNamespace

    import verl.utils.debug.metrics as dm

    g = torch.Generator().manual_seed(63)
    cases, arrays = [], {}
    for ci, (B, P, R, key) in enumerate([(6, 5, 12, "response_mask"), (4, 3, 9, "attention_mask")]):
        old = -torch.rand(B, R, generator=g) * 4
        roll = old + torch.randn(B, R, generator=g) * 0.05
        lens = torch.randint(1, R + 1, (B,), generator=g)
        rmask = (torch.arange(R)[None, :] < lens[:, None]).to(torch.int64)
        roll = torch.where(rmask.bool(), roll, torch.full_like(roll, -1.0))
        batch = {"rollout_log_probs": roll, "old_log_probs": old, "responses": torch.zeros(B, R, dtype=torch.int64)}
        if key == "response_mask":
            batch["response_mask"] = rmask
        else:
            batch["attention_mask"] = torch.cat([torch.ones(B, P, dtype=torch.int64), rmask], -1)
        out = dm.calculate_debug_metrics(SimpleNamespace(batch=batch))
        for k, v in batch.items():
            arrays[f"c{ci}_{k}"] = v
        cases.append({"mask_key": key, "metrics": {k: float(v) for k, v in out.items()}})
    _save("debug_metrics.npz", arrays, {"cases": cases, "ref": "verl/utils/debug/metrics.py:63-108"})


if __name__ == "__main__":
    which = sys.argv[1:] or ["ppo_loss", "masked_mean", "grpo", "gae", "logprob", "fused_linear", "masks", "tiny_qwen2"]
    for w in which:
        globals()[f"gen_{w}"]()
