"""Rollout engine: HFRollout semantics (verl/workers/rollout/hf_rollout.py:39-177) on our own decode loop.

Prefill of the left-padded prompts into a preallocated KV cache, then one decode step per response token
whose token selection (greedy / temperature sampling, EOS -> pad for finished rows) is the HIP kernel K4
writing straight into the ``responses`` column. Outputs match HFRollout's keys and post-processing:
``prompts, responses, input_ids, attention_mask, position_ids`` with responses padded to response_length,
position ids continuing from the last prompt position and the response attention mask from the first EOS.
The actor's bf16 compute buffer is read directly: no weight resharding between training and rollout.
"""

from __future__ import annotations

import gc
import time

import torch

from . import native
from .protocol import DataProto, TensorBatch
from .qwen2 import KVCache, KVCacheRows, PackedDecode, Qwen2Model
from .torch_functional import get_response_mask


_CAPTURE_STREAM = None


def capture_graph(body, pool):
    """Capture ``body()`` into a new HIP graph whose allocations come from the private pool ``pool``.

    This is torch.cuda.graph without its ``torch.cuda.empty_cache()`` on entry: that call handed every cached
    block of the step (~130 GB at config #2) back to the driver once per rollout, so the next stages re-allocated
    them (160 device allocations per step, each cleared by the driver before first use) and the old log-prob pass
    after the rollout ran up to 3x slow. The pool is the rollout's own and outlives each graph (the caller keeps
    the previous graph until the next one is captured), so its blocks are reused capture after capture."""
    global _CAPTURE_STREAM
    if _CAPTURE_STREAM is None:
        _CAPTURE_STREAM = torch.cuda.Stream()
    # no garbage collection during the capture: an unreachable CUDAGraph (or event) destroyed by a collection inside
    # it is a HIP call the capturing stream forbids, and the process aborts (seen in the GPU suite: a collection in
    # the middle of a decode-lane capture). torch.cuda.graph runs a full gc.collect() before capturing instead; here
    # that cost 45-75 ms per rollout (a large Python heap), so collection is only paused for the capture
    #
    # Refcount-driven destruction is not covered by pausing the collector: body() must not drop the last reference to
    # a CUDAGraph, an event or a stream. Audit of the bodies (round 6): the decode step bodies allocate tensors from
    # the graph pool and free temporaries (allocator bookkeeping, no HIP call); every workspace they reach is sized
    # before the capture and never replaced inside it (native._linear_workspace / _select_workspace raise instead);
    # the previous graph is released by the caller only after this capture ends (MI355XRollout._capture). The one
    # object the lanes body used to destroy inside the capture — the torch Event behind each Stream.wait_stream —
    # is now created before the capture and kept alive past it (MI355XRollout._decode_graphed_lanes).
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with gc_paused():
        with torch.cuda.stream(_CAPTURE_STREAM):
            graph.capture_begin(pool=pool)
            try:
                body()
            finally:
                graph.capture_end()
    return graph


class gc_paused:
    """Python's cyclic collector off inside the block, restored on exit (also on an exception) to what it was."""

    def __enter__(self):
        self.enabled = gc.isenabled()
        gc.disable()
        return self

    def __exit__(self, *exc):
        if self.enabled:
            gc.enable()
        return False


def replay_graph(graph, n):
    """``n`` replays of a captured step with the collector paused: a pause of the launching thread drains the device
    queue (4 ms idle stretches inside the decode in the kernel trace)."""
    with gc_paused():
        for _ in range(n):
            graph.replay()


class MI355XRollout:
    def __init__(self, module: Qwen2Model, config, dp_rank: int = 0):
        self.module = module
        self.config = config
        self.dp_rank = dp_rank
        self.calls = 0
        self._graph_pool = None  # private memory pool of the captured decode step, kept across rollouts
        self._graph = None  # the last captured decode step (released when the next one is captured)

    def _capture(self, body):
        if self._graph_pool is None:
            self._graph_pool = torch.cuda.graph_pool_handle()
        t0 = time.perf_counter()
        graph = capture_graph(body, self._graph_pool)
        self._graph = graph  # the previous graph goes only now, so the pool's use count never drops to zero
        self.last_capture_s = time.perf_counter() - t0  # host time of the capture (the device is idle meanwhile)
        return graph

    def generate_sequences(self, prompts: DataProto) -> DataProto:
        """hf_rollout.py:45-51: optional micro-batching of the prompt batch."""
        n = len(prompts)
        mbs = self.config.get("micro_batch_size") or n
        chunks = prompts.chunk(max(n // mbs, 1)) if n > mbs else [prompts]
        outs = [self._generate_minibatch(p, i * len(chunks[0])) for i, p in enumerate(chunks)]
        self.calls += 1
        return DataProto.concat(outs) if len(outs) > 1 else outs[0]

    @torch.no_grad()
    def _generate_minibatch(self, prompts: DataProto, row_offset: int) -> DataProto:
        cfg = self.config
        mi = prompts.meta_info
        do_sample = mi.get("do_sample", cfg.do_sample)
        is_validate = mi.get("validate", False)
        temperature = mi.get("temperature", cfg.temperature)
        response_length = mi.get("response_length", cfg.response_length)
        top_p = mi.get("top_p", cfg.get("top_p", 1.0))
        top_k = max(0, mi.get("top_k", cfg.get("top_k", 0)))
        if is_validate and do_sample:
            vk = cfg.val_kwargs
            top_k, top_p, temperature = max(0, vk.top_k), vk.top_p, vk.temperature
        eos = mi["eos_token_id"]
        pad_token_id = mi["pad_token_id"]
        eos_list = eos if isinstance(eos, (list, tuple)) else [eos]

        idx = prompts.batch["input_ids"]
        attention_mask = prompts.batch["attention_mask"]
        position_ids = prompts.batch["position_ids"]
        B, P = idx.shape
        R = int(response_length)
        dev = idx.device
        m = self.module
        m.training = False
        cache = KVCache(m.cfg, B, P + R, dev, m.dtype)
        group = self._prompt_group(idx, attention_mask, position_ids)
        self.last_prompt_group = group
        t0 = time.perf_counter()
        if group > 1:  # each distinct prompt prefilled once, its KV shared by the group's samples
            Bu = B // group
            h = m.prefill(KVCacheRows(cache, 0, Bu), idx[::group].contiguous(), attention_mask[::group].contiguous(),
                          position_ids[::group].contiguous())
            cache.share_prompts(group, P)
            h = h.repeat_interleave(group, 0)
        else:
            h = m.prefill(cache, idx, attention_mask, position_ids)
        torch.cuda.synchronize()
        self.last_prefill_s = time.perf_counter() - t0
        responses = torch.empty(B, R, dtype=torch.int64, device=dev)
        unfinished = torch.ones(B, dtype=torch.int32, device=dev)
        eos_t = torch.tensor(eos_list, dtype=torch.int64, device=dev)
        stop_ids = None if cfg.get("ignore_eos", False) else eos_t
        last_pos = position_ids[:, -1]
        seed = int(cfg.get("seed", 0)) + 7919 * self.calls
        row_base = self.dp_rank * (1 << 32) + row_offset
        sel = dict(do_sample=do_sample and temperature > 0, temperature=temperature if do_sample else 1.0, top_k=top_k,
                   top_p=top_p, seed=seed, row_base=row_base, pad_token_id=pad_token_id, eos_ids=stop_ids,
                   unfinished=unfinished)
        # lm_head fused with K4 (csrc/fused_linear.hip, no logits written) measured slower than hipBLASLt's
        # lm_head + K4 at 64 and 512 rows (rollout 0.43 vs 0.38 s, 1.22 vs 1.20 s): opt-in
        fused = bool(cfg.get("fused_select", False))
        self._fused_select = fused
        # rollout.calculate_log_probs: log p of each selected token from the decode step's own logits, under the
        # temperature the actor's compute_log_prob divides by (rollout.temperature, ray_trainer.py:1281)
        rollout_lp = torch.empty(B, R, dtype=torch.float32, device=dev) if cfg.get("calculate_log_probs") else None
        self._lp = dict(logprob_temperature=float(cfg.temperature)) if rollout_lp is not None else {}
        m.select_tokens(h, responses[:, 0], fused=fused, step=0, **self._lp_col(rollout_lp, 0), **sel)
        if cfg.get("use_hip_graph", True) and R > 2:
            self._decode_graphed(cache, responses, last_pos, P, R, sel, rollout_lp)
        else:
            for t in range(1, R):
                h = m.decode_step(cache, responses[:, t - 1], last_pos + t)
                m.select_tokens(h, responses[:, t], fused=fused, step=t, **self._lp_col(rollout_lp, t), **sel)
        del cache
        seq = torch.cat([idx, responses], dim=-1)
        # hf_rollout.py:151-160: positions continue from the last prompt position; mask up to first EOS
        full_pos = torch.empty(B, P + R, dtype=torch.int64, device=dev)
        full_pos[:, :P] = position_ids
        native.response_position_ids_(full_pos, P)
        resp_mask = get_response_mask(responses, eos_list, dtype=attention_mask.dtype)
        tensors = {
            "prompts": idx,
            "responses": responses,
            "input_ids": seq,
            "attention_mask": torch.cat([attention_mask, resp_mask], dim=-1),
            "position_ids": full_pos,
        }
        if rollout_lp is not None:  # vllm_rollout_spmd.py:359-362: -1 past each response
            tensors["rollout_log_probs"] = torch.where(resp_mask.bool(), rollout_lp, rollout_lp.new_full((), -1.0))
        return DataProto(batch=TensorBatch(tensors, batch_size=B))

    def _prompt_group(self, idx, attention_mask, position_ids):
        """Rows in runs of ``rollout.n`` identical prompts — the trainer's repeat(n, interleave=True) of the batch
        (ray_trainer.py:1146) — are prefilled once per distinct prompt and decode against one copy of its keys:
        the prefix caching the reference's vLLM rollout runs with (vllm_rollout_spmd.py:195,
        enable_prefix_caching=True). Same tokens as prefilling every row: the rows' prompt keys / values are
        identical. ``rollout.enable_prefix_caching`` False, another layout, or row lanes: 1 (every row its own)."""
        cfg = self.config
        n = int(cfg.get("n", 1) or 1)
        B = idx.shape[0]
        if n <= 1 or B % n or not cfg.get("enable_prefix_caching", True) or int(cfg.get("decode_lanes", 1) or 1) > 1:
            return 1
        same = torch.stack([(t.reshape(B // n, n, -1) == t.reshape(B // n, n, -1)[:, :1]).all()
                            for t in (idx, attention_mask, position_ids)]).all()
        return n if bool(same) else 1

    def _lp_col(self, rollout_lp, t):
        return dict(self._lp, logprob_out=rollout_lp[:, t]) if rollout_lp is not None else {}

    def _decode_graphed(self, cache, responses, last_pos, P, R, sel, rollout_lp=None):
        """Response tokens 1..R-1 as replays of ONE captured decode step.

        The step's only changing inputs live in device memory: the step counter t (token t-1 is read from
        ``responses``, written at cache position P+t-1, rotated at position last_pos+t; token t is selected
        into ``responses[:, t]`` with Philox offset t), so ~270 kernel launches per token become one graph
        launch and the host never waits on the device inside the loop. Step 1 runs eagerly (warms the GEMM
        heuristics for the decode shapes, outside capture); the captured body advances t itself."""
        m = self.module
        t_dev = torch.ones(1, dtype=torch.int64, device=responses.device)
        B = responses.shape[0]
        max_rows = int(self.config.get("packed_decode_max_rows", 512))
        lanes = self._decode_lanes(B, max_rows) if rollout_lp is None and cache.group == 1 else 1
        if lanes > 1:
            return self._decode_graphed_lanes(cache, responses, last_pos, P, R, sel, lanes)
        use = self.config.get("packed_decode", True) and PackedDecode.supported(m, B, max_rows)
        packed = PackedDecode(m, B, fused_norm=self.config.get("decode_fused_norm", False),
                              lm_head=self.config.get("decode_lm_head", True)) if use else None
        self.last_packed_decode = packed is not None

        prologue = packed is not None and m.store.w("embed_tokens").dtype == torch.bfloat16 and \
            self.config.get("decode_prologue", True)
        last_pos_flat = last_pos.reshape(-1).contiguous()

        lfn = packed.logits if packed is not None else None

        def body():
            if prologue:  # one launch: embedding, positions, cache slot, key_valid, t_cur, t_dev += 1
                h = packed.step_from(cache, responses, t_dev, last_pos_flat, P)
                m.select_tokens(h, responses[:, 0], fused=self._fused_select, step=0, dev_step=packed.t_cur,
                                logits_fn=lfn, **self._lp_col(rollout_lp, 0), **sel)
                return
            tok = responses.index_select(1, t_dev - 1)
            if packed is not None:
                h = packed.step(cache, tok, last_pos + t_dev, t_dev + (P - 1))
            else:
                h = m.decode_step_dev(cache, tok, last_pos + t_dev, t_dev + (P - 1))
            m.select_tokens(h, responses[:, 0], fused=self._fused_select, step=0, dev_step=t_dev,
                            logits_fn=lfn if packed is not None else None, **self._lp_col(rollout_lp, 0), **sel)
            t_dev.add_(1)

        body()  # t = 1, eager
        graph = self._capture(body)
        replay_graph(graph, max(0, R - 2))  # tokens 2 .. R - 1
        del graph, packed

    def _decode_lanes(self, B, max_rows):
        """Row lanes of the graphed decode step (config ``decode_lanes``): the rows split into equal groups of
        whole 32-row blocks, each group's decode step on its own stream of one graph. Every per-token kernel is
        row-independent (per-row attention, per-row GEMM outputs, per-row selection), so the lanes compute the
        same tokens as one B-row step; their latency-bound kernels overlap instead of running back to back."""
        m = self.module
        lanes = int(self.config.get("decode_lanes", 1) or 1)
        if lanes <= 1 or B % (32 * lanes) != 0:
            return 1
        if not (self.config.get("packed_decode", True) and self.config.get("decode_prologue", True)
                and m.store.w("embed_tokens").dtype == torch.bfloat16
                and PackedDecode.supported(m, B // lanes, max_rows)):
            return 1
        return lanes

    def _decode_graphed_lanes(self, cache, responses, last_pos, P, R, sel, lanes):
        """_decode_graphed over ``lanes`` row groups: lane j owns rows [j * B / lanes, (j + 1) * B / lanes) — its
        KV-cache rows, responses rows, step counter, PackedDecode buffers (the packed weights are shared) and
        workspaces (native.workspace_lane) — and its step is captured on its own stream, forked from and joined
        to the capture stream, so one replay runs all lanes' steps concurrently. Sampling stays row-identical:
        lane j's Philox rows start at row_base + j * B / lanes."""
        m = self.module
        B = responses.shape[0]
        rows = B // lanes
        dev = responses.device
        last_pos_flat = last_pos.reshape(-1).contiguous()
        lane_state = []
        shared_w = None
        for j in range(lanes):
            r0, r1 = j * rows, (j + 1) * rows
            pk = PackedDecode(m, rows, weights=shared_w, fused_norm=self.config.get("decode_fused_norm", False),
                              lm_head=False)
            shared_w = pk.w
            sel_j = dict(sel, row_base=sel["row_base"] + r0, unfinished=sel["unfinished"][r0:r1])
            lane_state.append(dict(cache=KVCacheRows(cache, r0, r1), resp=responses[r0:r1], pk=pk, sel=sel_j,
                                   last_pos=last_pos_flat[r0:r1].contiguous(),
                                   t_dev=torch.ones(1, dtype=torch.int64, device=dev)))
        self.last_packed_decode = True

        def body(j):
            st = lane_state[j]
            with native.workspace_lane(j):
                h = st["pk"].step_from(st["cache"], st["resp"], st["t_dev"], st["last_pos"], P)
                m.select_tokens(h, st["resp"][:, 0], fused=self._fused_select, step=0, dev_step=st["pk"].t_cur,
                                **st["sel"])

        for j in range(lanes):  # t = 1, eager (sizes every lane's workspaces outside capture)
            body(j)
        side = [torch.cuda.Stream(device=dev) for _ in range(lanes - 1)]
        # the fork / join events exist before the capture and outlive it (Stream.wait_stream would create and destroy
        # one per call inside the capture)
        fork = torch.cuda.Event()
        joins = [torch.cuda.Event() for _ in side]

        def lanes_body():
            main = torch.cuda.current_stream()
            fork.record(main)
            for s in side:
                s.wait_event(fork)
            body(0)
            for j, s in enumerate(side, start=1):
                with torch.cuda.stream(s):
                    body(j)
            for s, ev in zip(side, joins):
                ev.record(s)
                main.wait_event(ev)

        graph = self._capture(lanes_body)
        replay_graph(graph, max(0, R - 2))
        del graph, lane_state, fork, joins
