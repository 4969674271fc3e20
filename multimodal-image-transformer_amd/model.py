"""ImageToTextModel: frozen vision encoder + projection + Transformer decoder (reference model.py:12-255).

Drop-in surface:
  * ``ImageToTextModel(decoder_vocab_size, decoder_embed_dim, decoder_heads, decoder_layers,
    decoder_ff_dim, decoder_max_seq_len, decoder_dropout, decoder_pad_idx)`` (model.py:14-16), the
    encoder chosen by config.ENCODER_MODEL_NAME;
  * ``forward(image_tensors f32[B,3,H,W], tgt_tokens i64[B,T]) -> f32[B,T,V]`` (model.py:116-169);
  * ``generate(image, start_token_id, end_token_id, max_len=100, method='greedy', beam_size=3)``
    (model.py:171-255);
  * ``state_dict()`` / ``load_state_dict()`` in the reference's key names.
Added for the MI355X path:
  * ``train_step(images, decoder_input_tokens, target_tokens, dist=None)``: the whole of
    train.py:75-93 (forward, CE(ignore PAD), backward) as one kernel sequence with no host sync,
    returning the loss as a device scalar; ``optim.AdamW.step(clip)`` finishes train.py:96-100.
  * ``memory_mode`` "cls" (reference: CLS token only, model.py:141) or "patches" (north star:
    cross-attention over the projected patch sequence).
"""
from __future__ import annotations

import math
import os
from collections import OrderedDict
from typing import Dict, Iterator, List, Optional, Tuple

import torch

import config
import data
import native
from decoder import TransformerDecoder, decoder_entries, flat_to_reference, reference_to_flat
from encoder import VisionEncoder, build_encoder
from params import FlatParams

def _dtype_from_config(dtype):
    if dtype is None:
        dtype = config.DTYPE
    if isinstance(dtype, torch.dtype):
        return dtype
    return {"bf16": torch.bfloat16, "bfloat16": torch.bfloat16, "fp32": torch.float32, "float32": torch.float32}[dtype]


# encoder chunks (VisionEncoder.forward_iter: patch embedding, layers, final LayerNorm) of the prefetched
# next batch issued before the decoder's first launch (train step); 0 / 1 / 2 / 4 / all measured within
# 0.3 % of each other
ENC_LEAD = 1

class GraphedStep:
    """A captured train step. step(images, decoder_input_tokens, target_tokens) copies a batch into
    the static buffers (skip by passing nothing) and replays; returns the loss device scalar. The
    learning rate is a device scalar the graph reads, refreshed from optimizer.param_groups before
    every replay (a scheduler's change takes effect like in the eager loop)."""

    def __init__(self, graph, images, dec_in, targets, loss, optimizer=None):
        self.graph, self.images, self.dec_in, self.targets, self.loss = graph, images, dec_in, targets, loss
        self.optimizer = optimizer

    def __call__(self, images=None, decoder_input_tokens=None, target_tokens=None):
        if images is not None:
            self.images.copy_(images, non_blocking=True)
            self.dec_in.copy_(decoder_input_tokens, non_blocking=True)
            self.targets.copy_(target_tokens, non_blocking=True)
        if self.optimizer is not None:
            self.optimizer._sync_lr()
        self.graph.replay()
        return self.loss


class ImageToTextModel:
    def __init__(self, decoder_vocab_size: int, decoder_embed_dim: int, decoder_heads: int, decoder_layers: int,
                 decoder_ff_dim: int, decoder_max_seq_len: int, decoder_dropout: float, decoder_pad_idx: int, *,
                 encoder: Optional[VisionEncoder] = None, memory_mode: Optional[str] = None, dtype=None, device=None,
                 seed: Optional[int] = None):
        native.require_gpu()
        native.load_library()
        self.device = torch.device(device) if device is not None else torch.device("cuda", torch.cuda.current_device())
        self.dtype = _dtype_from_config(dtype)
        seed = config.RANDOM_SEED if seed is None else seed
        self.encoder = encoder if encoder is not None else build_encoder(device=self.device, dtype=self.dtype,
                                                                          seed=seed)
        if self.encoder.dtype != self.dtype:
            raise ValueError("encoder and model compute dtypes differ")
        self.memory_mode = memory_mode or config.MEMORY_MODE
        if self.memory_mode not in ("cls", "patches"):
            raise ValueError(f"memory_mode must be 'cls' or 'patches', got {self.memory_mode}")
        self.encoder.configure_for(self.memory_mode)  # residual-stream precision for this memory (encoder.py)
        self.encoder_output_dim = self.encoder.hidden_size
        self.decoder_embed_dim = decoder_embed_dim
        self.decoder_pad_idx = decoder_pad_idx
        E, d = self.encoder_output_dim, decoder_embed_dim
        self.has_projection = E != d  # model.py:97-102: Linear if dims differ, else Identity
        self.store = FlatParams(decoder_entries(decoder_vocab_size, d, decoder_layers, decoder_ff_dim,
                                                E if self.has_projection else None), self.device, self.dtype)
        self.store.vocab = decoder_vocab_size
        # what optim.AdamW needs to speak torch.optim.AdamW's state_dict in the reference's parameter
        # order (frozen encoder tensors first: model.py:48-66 registers the encoder before the rest)
        self.store.layout = dict(V=decoder_vocab_size, d=d, L=decoder_layers, F=decoder_ff_dim,
                                 proj_in=E if self.has_projection else None,
                                 n_encoder_params=self.encoder.num_reference_params())
        self.decoder = TransformerDecoder(decoder_vocab_size, d, decoder_heads, decoder_layers, decoder_ff_dim,
                                          decoder_max_seq_len, decoder_dropout, decoder_pad_idx, store=self.store,
                                          device=self.device)
        self.decoder.init_weights(seed + 1)
        if self.has_projection:
            g = torch.Generator().manual_seed(seed + 2)
            b = 1.0 / math.sqrt(E)  # nn.Linear default init bounds
            self.store.p("projection.weight").copy_((torch.rand(d, E, generator=g) * 2 - 1) * b)
            self.store.p("projection.bias").copy_((torch.rand(d, generator=g) * 2 - 1) * b)
            self.store.sync_shadow()
        # the processor the encoder was trained with (model.py:69-83 loads AutoImageProcessor for the
        # encoder's name): ViT = bilinear resize + mean/std 0.5; CLIP = shortest-edge bicubic resize,
        # centre crop, CLIP mean/std — bit-identical to the HF processors (tests/test_data_*.py)
        self.image_processor = data.ImagePreprocessor(self.encoder.kind, self.encoder.image, self.device)
        self.training = True
        # dropout RNG state: a device counter (graph-replay safe), distinct per DP rank
        self.seed_t = torch.tensor([seed * 1000003], dtype=torch.int64, device=self.device)
        self._mem: Dict[tuple, torch.Tensor] = {}
        self._enc_stream = None
        self._enc_slot = 0
        self._prefetched = None
        self._slot_free = None           # native.HipEvents(2): end of the backward of the step that read slot i
        self._slot_freed = [False, False]  # slot i's event recorded since the slot was last read
        self._params: Optional["OrderedDict[str, torch.nn.Parameter]"] = None
        self._gen = 0  # bumped by every forward that writes the shared arenas (autograd staleness check)

    # --- nn.Module-like surface ----------------------------------------------------------------
    def train(self, mode: bool = True):
        self.training = mode
        self.decoder.train(mode)
        return self

    def eval(self):
        return self.train(False)

    def to(self, device):
        if torch.device(device).type != self.device.type:
            raise ValueError("ImageToTextModel lives on the GPU it was built on")
        return self

    def _param_table(self) -> "OrderedDict[str, torch.nn.Parameter]":
        """One nn.Parameter per trainable flat entry, ALIASING the f32 master buffer (same storage
        and version counter): torch.optim.AdamW / clip_grad_norm_ update and read the very memory
        the kernels use; .grad is a view of the flat gradient buffer once a backward ran."""
        if self._params is None:
            self._params = OrderedDict((n, torch.nn.Parameter(self.store.p(n), requires_grad=True))
                                       for n in self.store.names())
            for n, p in self._params.items():
                p._mit_store = self.store  # optim.AdamW(model.parameters()) finds the flat buffers
                p.register_post_accumulate_grad_hook(self._grad_to_flat(n))
        return self._params

    def _grad_to_flat(self, name):
        """After autograd accumulated a parameter's gradient (model(images, tokens) -> loss.backward()):
        make p.grad the view of the flat gradient buffer (one copy when autograd created a new tensor),
        so clip_grad_norm_, torch.optim.AdamW, the fused optim.AdamW and the DP buckets all see it."""
        st = self.store

        def hook(p):
            g = st.g(name)
            if p.grad is not None and p.grad.data_ptr() != g.data_ptr():
                g.copy_(p.grad)
                p.grad = g
        return hook

    def parameters(self, recurse: bool = True) -> Iterator[torch.nn.Parameter]:
        """The trainable parameters (projection + decoder; the encoder is frozen, model.py:87-90)
        in flat-buffer order. Padded entries (the vocabulary head, decoder.padded_vocab) include
        their zero pad rows, which get exactly-zero gradients."""
        return iter(self._param_table().values())

    def named_parameters(self, prefix: str = "", recurse: bool = True) -> Iterator[Tuple[str, torch.nn.Parameter]]:
        for n, p in self._param_table().items():
            yield prefix + n, p

    def zero_grad(self, set_to_none: bool = True):
        for p in self._param_table().values():
            if set_to_none:
                p.grad = None
            elif p.grad is not None:
                p.grad.zero_()

    def num_trainable(self) -> int:
        return sum(n for _, _, _, n in self.store.entries)

    def set_rank_seed(self, rank: int, seed: Optional[int] = None):
        """Dropout streams differ per data-parallel rank."""
        seed = config.RANDOM_SEED if seed is None else seed
        self.seed_t.fill_(seed * 1000003 + rank * 7919 * 65537)

    # --- memory (encoder -> projection) ----------------------------------------------------------
    def _encoder_rows(self, images: torch.Tensor, slot: int = 0):
        """Frozen encoder -> (enc_rows, enc_ld, S): the rows that feed the projection."""
        self.encoder.configure_for(self.memory_mode)  # memory_mode may have changed since __init__ (cheap)
        B = images.shape[0]
        N, E = self.encoder.N, self.encoder.E
        if self.memory_mode == "cls":
            enc = self.encoder.forward(images, rows="cls", slot=slot)  # [B, E] view, row stride N*E
            return enc, N * E, 1
        enc = self.encoder.forward(images, rows="all", slot=slot)  # [B, N, E]
        return enc.reshape(B * N, E), E, N

    def _encoder_rows_iter(self, images: torch.Tensor, slot: int = 0):
        """_encoder_rows as a generator of launch chunks (VisionEncoder.forward_iter)."""
        self.encoder.configure_for(self.memory_mode)
        B = images.shape[0]
        N, E = self.encoder.N, self.encoder.E
        if self.memory_mode == "cls":
            enc = yield from self.encoder.forward_iter(images, rows="cls", slot=slot)
            return enc, N * E, 1
        if self.encoder.groups_for(B) == 2:  # CLIP-L towers at B = 64: two image groups on two streams
            enc = yield from self.encoder.forward_iter_groups(images, slot)
        else:
            enc = yield from self.encoder.forward_iter(images, rows="all", slot=slot)
        return enc.reshape(B * N, E), E, N

    def prefetch_encoder(self, images: torch.Tensor):
        """Start the frozen encoder's forward for the NEXT batch on a second stream; the next
        train_step(images) consumes it instead of recomputing. The encoder has no trainable state, so
        its output does not depend on the step in between: the result is identical, and its GEMMs
        fill the CUs the decoder's small kernels leave idle. Double-buffered arenas (slot 0/1)."""
        for _ in self.prefetch_encoder_iter(images):
            pass

    def prefetch_encoder_iter(self, images: torch.Tensor):
        """prefetch_encoder as a generator: each next() issues one launch chunk of the encoder forward
        (the patch embedding, one layer, the final LayerNorm) on the encoder stream. The train step
        interleaves the chunks with its decoder layers, so neither stream's launches wait behind the
        other's on the host (launches issue in program order, ~3.6 us each from a replayed plan)."""
        if self._enc_stream is None:
            self._enc_stream = torch.cuda.Stream(device=self.device)
            self._enc_events = native.HipEvents(8)
        slot = 1 - self._enc_slot
        images = images.to(self.device, non_blocking=True)
        enc = self._enc_stream.cuda_stream
        # the arena's previous reader (two steps back) is done: the encoder stream waits for the end of
        # that step's backward (its last read: the projection weight gradient; the encoder then runs
        # beside that step's HBM-bound clip + AdamW: +0.2 %), or for everything on main (the autograd
        # path records no slot event)
        if self._slot_freed[slot]:
            native.HipEvents.wait(enc, self._slot_free.pool[slot])
        else:
            self._enc_events.wait_stream(enc, native.stream_ptr())
        it = self._encoder_rows_iter(images, slot)
        while True:
            with torch.cuda.stream(self._enc_stream):  # (never left entered across a yield)
                try:
                    next(it)
                except StopIteration as e:
                    out = e.value
                    break
            yield
        ev = self._enc_events.record(enc)
        self._prefetched = (images, slot, out, ev)

    def _take_encoded(self, images: torch.Tensor):
        """The encoder rows for images: the prefetched ones when they are for these images (this stream
        waits for them), else computed here into the current arena."""
        pf, self._prefetched = self._prefetched, None
        if pf is not None and pf[0].data_ptr() == images.data_ptr() and pf[0].shape == images.shape:
            _, self._enc_slot, (enc_rows, enc_ld, S), ev = pf
            native.HipEvents.wait(native.stream_ptr(), ev)
            out = enc_rows, enc_ld, S
        else:
            out = self._encoder_rows(images, self._enc_slot)
        # the slot is being read again: a later prefetch into it must wait for this reader (re-armed by
        # _train_step once the step's readers are issued; every other caller leaves it unarmed, so the
        # prefetch waits for everything on the main stream)
        self._slot_freed[self._enc_slot] = False
        return out

    def _encode_memory(self, images: torch.Tensor, refresh: bool = True):
        """Returns (mem_rows, mem_ld, S, enc_rows, enc_ld): memory [B*S rows of d] and the
        encoder features that feed the projection (for its weight gradient). refresh: re-cast the
        bf16 weight shadow unconditionally (every path but the fused train step: params.ensure_shadow)."""
        B = images.shape[0]
        E, d = self.encoder.E, self.decoder_embed_dim
        self.store.ensure_shadow(force=refresh)
        self._gen += 1
        enc_rows, enc_ld, S = self._take_encoded(images)
        if not self.has_projection:
            return enc_rows, enc_ld, S, enc_rows, enc_ld
        key = (B, S)
        if key not in self._mem:
            self._mem[key] = torch.empty(B * S, d, dtype=self.dtype, device=self.device)
        mem = self._mem[key]
        native.gemm(enc_rows, self.store.w("projection.weight"), mem, B * S, d, E, lda=enc_ld,
                    bias=self.store.p("projection.bias"))
        return mem, d, S, enc_rows, enc_ld

    # --- forward (model.py:116-169) ------------------------------------------------------------
    def forward(self, image_tensors: torch.Tensor, tgt_tokens: torch.Tensor) -> torch.Tensor:
        """f32 logits [B, T, V]. With grad enabled and trainable parameters, the result carries an
        autograd node whose backward runs the HIP backward (the reference's loss.backward(),
        train.py:93); otherwise a forward-only launch sequence."""
        if torch.is_grad_enabled() and any(p.requires_grad for p in self._param_table().values()):
            return self._forward_ops(image_tensors, tgt_tokens)
        images = image_tensors.to(self.device)
        tokens = tgt_tokens.to(self.device, torch.int64).contiguous()
        B, T = tokens.shape
        mem, mem_ld, S, _, _ = self._encode_memory(images)
        A = self.decoder.acts(B, T, S, False)
        out = torch.empty(B * T, self.decoder.Vp, dtype=torch.float32, device=self.device)
        p = self.decoder.dropout if self.training else 0.0
        if p > 0:
            native.step_inc(self.seed_t)
        self.decoder.run_forward(tokens, mem, mem_ld, S, A, self.seed_t, False, logits_out=out, drop_p=p)
        return self.decoder.unpad_logits(out, B, T)

    __call__ = forward

    def _forward_ops(self, image_tensors, tgt_tokens):
        """model(images, tokens) under autograd (the reference loop, train.py:80-100): the frozen encoder
        runs as usual (no gradient), the projection and the decoder as torch.ops.mit_hip operators
        (ops.py, decoder.forward_ops) whose registered backward formulas run the HIP backward kernels.
        Parameter gradients land in the flat gradient buffer (see _param_table's hooks)."""
        import ops
        mh = ops.load()
        images = image_tensors.to(self.device)
        tokens = tgt_tokens.to(self.device, torch.int64).contiguous()
        B, T = tokens.shape
        self.store.ensure_shadow(force=True)
        self._gen += 1
        enc_rows, enc_ld, S = self._take_encoded(images)
        E = self.encoder_output_dim
        # the encoder arena is reused by the next forward: the projection's saved input is a copy
        enc = torch.as_strided(enc_rows, (B * S, E), (enc_ld, 1)).clone()
        P = self._param_table()
        p = self.decoder.dropout if self.training else 0.0
        seed = None
        if p > 0:
            native.step_inc(self.seed_t)
            seed = self.seed_t.clone()  # the backward regenerates this forward's masks whatever runs between
        if self.has_projection:
            st = self.store
            mem = mh.linear(enc, P["projection.weight"], P["projection.bias"],
                            weight_lp=st.w("projection.weight") if st.shadow is not st.master else None)
        else:
            mem = enc
        return self.decoder.forward_ops(tokens, mem, S, P, seed, p)

    # --- fused train step (train.py:75-93) -----------------------------------------------------
    def train_step(self, images: torch.Tensor, decoder_input_tokens: torch.Tensor, target_tokens: torch.Tensor,
                   dist=None, next_images: Optional[torch.Tensor] = None) -> torch.Tensor:
        """See _train_step. (Stream priorities for the step's own streams over the encoder prefetch
        measured neutral to -1.7 %, DESIGN.md §4.1c: all streams run at the default priority.)"""
        return self._train_step(images, decoder_input_tokens, target_tokens, dist, next_images)

    def _train_step(self, images: torch.Tensor, decoder_input_tokens: torch.Tensor, target_tokens: torch.Tensor,
                    dist=None, next_images: Optional[torch.Tensor] = None) -> torch.Tensor:
        """Forward + CE(ignore PAD, mean over the GLOBAL non-PAD count) + backward into the flat
        gradient buffer. Returns the loss as a device scalar [1] (no host sync).
        next_images: the next batch's images, whose (frozen) encoder forward then runs on a second
        stream beside this step's decoder work (prefetch_encoder); results are unchanged."""
        images = images.to(self.device, non_blocking=True)
        tokens = decoder_input_tokens.to(self.device, torch.int64, non_blocking=True).contiguous()
        targets = target_tokens.to(self.device, torch.int64, non_blocking=True).contiguous()
        B, T = tokens.shape
        mem, mem_ld, S, enc_rows, enc_ld = self._encode_memory(images, refresh=False)
        pf = self.prefetch_encoder_iter(next_images) if next_images is not None else None

        def tick(n=1):
            nonlocal pf
            while pf is not None and n > 0:
                if next(pf, tick) is tick:  # exhausted: the prefetch is fully issued
                    pf = None
                n -= 1
        # the next batch's encoder: ENC_LEAD chunks now, then one per decoder layer (forward and backward),
        # the rest after the backward
        tick(ENC_LEAD)
        dec = self.decoder
        A = dec.acts(B, T, S, True)
        native.step_inc(self.seed_t)
        logits, _ = dec.run_forward(tokens, mem, mem_ld, S, A, self.seed_t, True, tick=tick)
        native.zero(A.count_loss)
        native.count_targets(targets, self.decoder_pad_idx, A.count)
        if dist is not None:
            dist.all_reduce_count(A.count)
        native.cross_entropy(logits, targets, self.decoder_pad_idx, A.count, A.loss_sum, True, row_loss=A.row_loss,
                             V=dec.V, ld=dec.Vp)
        proj = (enc_rows, enc_ld, self.encoder_output_dim) if self.has_projection else None
        dec.run_backward(tokens, mem, mem_ld, S, A, self.seed_t, logits, proj_input=proj,
                         grads_ready=dist.grads_ready if dist is not None else None, tick=tick)
        tick(1 << 30)
        if self._enc_stream is not None:  # this step's last reader of its encoder slot is issued
            if self._slot_free is None:
                self._slot_free = native.HipEvents(2)
            self._slot_free.record_at(self._enc_slot, native.stream_ptr())
            self._slot_freed[self._enc_slot] = True
        native.scalar_div(A.loss_sum, A.count, A.loss)
        if dist is not None:
            dist.finish_backward(A.loss)
        return A.loss

    def make_graphed_step(self, optimizer, images, decoder_input_tokens, target_tokens, max_norm: float):
        """Capture train_step + optimizer.step(max_norm) (train.py:75-100, ~300 kernel launches) into
        ONE hipGraph over static input buffers. The two warm-up executions that size the arenas
        are undone (parameters, AdamW state and counters restored) before capture, so the graph
        starts from the same state the model had. Returns a GraphedStep (call it per batch)."""
        dev = self.device
        st_img = images.to(dev).clone()
        st_in = decoder_input_tokens.to(dev, torch.int64).clone()
        st_tg = target_tokens.to(dev, torch.int64).clone()
        store = self.store
        store.ensure_optimizer_state()
        saved = [t.clone() for t in (store.master, store.shadow, store.exp_avg, store.exp_avg_sq, optimizer.step_t,
                                     self.seed_t)]
        side = torch.cuda.Stream(device=dev)
        side.wait_stream(torch.cuda.current_stream(dev))
        with torch.cuda.stream(side):
            for _ in range(2):
                self.train_step(st_img, st_in, st_tg)
                optimizer.step(max_norm)
        torch.cuda.current_stream(dev).wait_stream(side)
        torch.cuda.synchronize(dev)
        for dst, src in zip((store.master, store.shadow, store.exp_avg, store.exp_avg_sq, optimizer.step_t,
                             self.seed_t), saved):
            dst.copy_(src)
        torch.cuda.synchronize(dev)
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            loss = self.train_step(st_img, st_in, st_tg)
            optimizer.step(max_norm)
        return GraphedStep(graph, st_img, st_in, st_tg, loss, optimizer)

    @torch.no_grad()
    def eval_loss(self, images, decoder_input_tokens, target_tokens) -> torch.Tensor:
        """train.py:141-145 (forward + CE) without materialising f32 logits; device scalar."""
        images = images.to(self.device)
        tokens = decoder_input_tokens.to(self.device, torch.int64).contiguous()
        targets = target_tokens.to(self.device, torch.int64).contiguous()
        B, T = tokens.shape
        mem, mem_ld, S, _, _ = self._encode_memory(images)
        A = self.decoder.acts(B, T, S, False)
        logits, _ = self.decoder.run_forward(tokens, mem, mem_ld, S, A, self.seed_t, False, drop_p=0.0)
        native.zero(A.count)
        native.zero(A.loss_sum)
        native.count_targets(targets, self.decoder_pad_idx, A.count)
        native.cross_entropy(logits, targets, self.decoder_pad_idx, A.count, A.loss_sum, False, row_loss=A.row_loss,
                             V=self.decoder.V, ld=self.decoder.Vp)
        native.scalar_div(A.loss_sum, A.count, A.loss)
        return A.loss

    # --- generate (model.py:171-255) -----------------------------------------------------------
    @torch.no_grad()
    def generate(self, image, start_token_id, end_token_id, max_len=100, method="greedy", beam_size=3) -> List[int]:
        if method == "beam":
            print("Beam search not fully implemented in this example. Falling back to greedy.")
            method = "greedy"
        if method != "greedy":
            raise ValueError(f"Unsupported generation method: {method}. Choose 'greedy' or 'beam'.")
        self.eval()
        if isinstance(image, torch.Tensor):
            pv = image if image.dim() == 4 else image.unsqueeze(0)
        else:
            pv = self.image_processor(images=image, return_tensors="pt")["pixel_values"]
        pv = pv.to(self.device).float()
        mem, mem_ld, S, _, _ = self._encode_memory(pv)
        mem3 = mem.view(1, S, -1) if mem_ld == self.decoder_embed_dim else None
        if mem3 is None:  # identity projection + cls: gather the strided row
            mem3 = mem[:1].reshape(1, 1, -1).contiguous()
        ids = [int(start_token_id)]
        for _ in range(max_len - 1):
            logits = self.decoder.forward(torch.tensor([ids], device=self.device), mem3)
            nxt = int(torch.argmax(logits[0, -1]).item())
            ids.append(nxt)
            if nxt == end_token_id:
                break
        return ids

    @torch.no_grad()
    def generate_batch(self, images, start_token_id: int, end_token_id: int, max_len: int = 100,
                       use_graph: bool = True, check_every: int = 8, streams: Optional[int] = None,
                       next_images: Optional[torch.Tensor] = None) -> List[List[int]]:
        """Greedy captions for a whole batch (BASELINE config 5): per image the same token list as
        generate() (model.py:171-242: START, argmax of the last position each step, stop after END,
        at most max_len ids), computed with cached self-attention K/V, the cross-attention K/V of
        the image memory computed once, and ONE hipGraph-captured step replayed per token. The host
        checks the finished count every `check_every` tokens (the only synchronisation).

        streams: the images are decoded as this many independent row groups, each with its own state,
        issued on its own HIP stream (default: env MIT_DECODE_STREAMS, else 1). Rows never interact in
        greedy decoding and every kernel computes a row the same way at any batch size, so the ids
        do not depend on the grouping. Measured at B = 256 (configs[4]): 2 / 3 / 4 groups take 1.12 /
        1.23 / 1.53x the one-group time -- the groups' kernels do overlap, but every kernel boundary
        costs the same whatever its size, so one group of full-width launches is fastest.

        next_images: the next call's images (pixel values on the device); their frozen encoder forward is
        issued on the encoder stream one launch chunk per token step, beside this call's latency-bound
        token steps, and the next call takes it (as train_step's next_images; the ids are unchanged)."""
        self.eval()
        pv = images if isinstance(images, torch.Tensor) else \
            self.image_processor(images=images, return_tensors="pt")["pixel_values"]
        pv = pv.to(self.device).float()
        B = pv.shape[0]
        mem, mem_ld, S, _, _ = self._encode_memory(pv)
        dec = self.decoder
        if streams is None:
            streams = int(os.environ.get("MIT_DECODE_STREAMS", "1"))
        G = max(1, min(int(streams), B))
        bounds = [B * i // G for i in range(G + 1)]
        states = [dec.decode_begin(mem[bounds[i] * S:bounds[i + 1] * S], mem_ld, S, bounds[i + 1] - bounds[i], max_len,
                                   start_token_id, end_token_id) for i in range(G)]
        steps = max_len - 1
        if steps > 0:
            for stt in states:
                dec.decode_step(stt)  # position 0 (eager: warms every kernel before capture)
            done = 1
            cur = torch.cuda.current_stream()
            side = [cur] + [torch.cuda.Stream(device=self.device) for _ in range(G - 1)]
            for s_ in side[1:]:
                s_.wait_stream(cur)

            def one_step():
                for stt, s_ in zip(states, side):
                    with torch.cuda.stream(s_):
                        dec.decode_step(stt)
            launch = os.environ.get("MIT_DECODE_LAUNCH", "plan") if use_graph else "eager"
            if launch == "graph" and steps > 1:
                # one hipGraph per group (ROCm launches a graph's nodes one by one from the host:
                # ~8.7 us each, so the groups' graphs hardly overlap)
                runs = []
                for stt in states:
                    graph = torch.cuda.CUDAGraph()
                    with torch.cuda.graph(graph):
                        dec.decode_step(stt)
                    runs.append(graph.replay)

                def run():
                    for r, s_ in zip(runs, side):
                        with torch.cuda.stream(s_):
                            r()
            elif launch == "plan" and steps > 1:
                # the step's launches recorded once (a real step) and re-issued from C++ (mit_plan_run,
                # ~3.6 us per launch), every group on its own stream
                prog = native.record(one_step)
                done += 1
                run = prog.run
            else:
                run = one_step
            pf = self.prefetch_encoder_iter(next_images) if next_images is not None else None
            while done < steps:
                n = min(check_every, steps - done)
                for _ in range(n):
                    run()
                    # one encoder chunk per token step (one per 3 or 6 steps measured the same)
                    if pf is not None and next(pf, pf) is pf:
                        pf = None
                done += n
                if sum(int(stt.n_finished.item()) for stt in states) == B:
                    break
            for _ in pf or ():
                pass
            for s_ in side[1:]:
                cur.wait_stream(s_)
        out = []
        for stt in states:
            out.extend(stt.token_lists())
        return out

    def sync_shadow(self):
        """Re-cast the bf16 weight shadow the kernels read from the f32 master. Needed only after
        editing weights out of band (through ``p.data``, which torch's version counter does not see)
        and before a fused ``train_step``; every other path refreshes the shadow itself
        (params.FlatParams.ensure_shadow)."""
        self.store.sync_shadow()

    # --- checkpoints (reference key names) --------------------------------------
    def state_dict(self) -> Dict[str, torch.Tensor]:
        sd = {}
        for k, v in self.encoder.hf_state_dict().items():
            sd["encoder." + k] = v
        if self.has_projection:
            sd["projection.weight"] = self.store.p("projection.weight").detach().clone()
            sd["projection.bias"] = self.store.p("projection.bias").detach().clone()
        sd.update(flat_to_reference(self.store, self.decoder.L, self.decoder_embed_dim))
        sd["decoder.positional_encoding.pe"] = self.decoder.pe.unsqueeze(0).clone()
        return sd

    def check_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        """Raise (KeyError / ValueError) unless sd loads into this model: every trainable tensor
        present (strict) with the reference shape, encoder keys (if any) loadable. Touches nothing."""
        from optim import reference_trainable
        ref_shapes = dict(reference_trainable(self.store.layout))
        missing = [k for k in ref_shapes if k not in sd]
        if strict and missing:
            raise KeyError(f"missing keys: {missing[:6]}{'...' if len(missing) > 6 else ''}")
        bad = [(k, tuple(sd[k].shape), s) for k, s in ref_shapes.items() if k in sd and tuple(sd[k].shape) != s]
        if bad:
            raise ValueError("shape mismatch (checkpoint vs model): " +
                             ", ".join(f"{k} {a} vs {b}" for k, a, b in bad[:4]))
        enc = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
        if enc:
            self.encoder.check_hf_state_dict(enc)

    def load_state_dict(self, sd: Dict[str, torch.Tensor], strict: bool = True):
        self.check_state_dict(sd, strict)
        enc = {k[len("encoder."):]: v for k, v in sd.items() if k.startswith("encoder.")}
        if enc:
            self.encoder.load_hf_state_dict(enc)
        flat = reference_to_flat(sd, self.decoder.L, self.decoder_embed_dim)
        names = set(self.store.names())
        with torch.no_grad():
            for k, v in flat.items():
                if k in names:
                    dst = self.store.p(k)
                    v = v.to(self.device, torch.float32)
                    if k.startswith("fc_out.") and v.shape[0] != dst.shape[0]:  # padded vocabulary head
                        if v.shape[0] != self.decoder.V:
                            raise ValueError(f"{k}: {tuple(v.shape)} does not match vocab {self.decoder.V}")
                        dst.zero_()
                        dst[:v.shape[0]].copy_(v)
                    else:
                        dst.copy_(v.reshape(dst.shape))
        self.store.sync_shadow()
        return self

    # --- accounting ----------------------------------------------------------------------------
    def flops_per_pair(self, T: int) -> float:
        """Algorithmic train FLOPs per image-caption pair: encoder fwd + 3 x decoder fwd
        (+ the projection, counted with the decoder as 3 x its forward)."""
        S = 1 if self.memory_mode == "cls" else self.encoder.N
        dec = self.decoder.flops_per_sequence(T, S)
        proj = 2 * S * self.encoder.E * self.decoder_embed_dim if self.has_projection else 0
        return self.encoder.flops_per_image() + 3 * (dec + proj)
