"""CadenceGemma model assembly on MI355X (inference only: no backward kernels,
so the entry points run under torch.no_grad()).

Reference: `recurrentgemma/torch/griffin.py` (`Griffin` :35-245).  Same
constructor / `forward(tokens, segment_pos, cache, return_logits,
return_cache, img_path)` / `init_cache(batch_size, dtype)` surface and
state-dict keys (`embedder.*`, `blocks.{i}.*`, `final_norm.scale`,
`vis_encoder.{dino,siglip}.*`, `projector.proj.*`).

Differences the reference cannot express:
  * real batches (Q5): `tokens [B, T]` rows are independent;
  * `images=[B,3,S,S]` pixels in [0,1] as the batched form of `img_path`;
  * n_vis = (S // 14)^2 instead of the hard-coded 729 (Q2).
The splice itself follows griffin.py:179-191 exactly: when the positions
contain a 0, the projected image tokens are placed in front of the text
(before BOS) and the positions become [0, 1, .., n_vis-1, text positions]
(Q1), i.e. image and text are separate documents.
"""

from __future__ import annotations

import torch
from torch import nn

from . import common, layers, modules, ops
from .tracing import trace
from .layers import _flat
from .vision import MLPProjector, VisionEncoder

Cache = dict[str, modules.ResidualBlockCache]


class Griffin(nn.Module):
  """Griffin LM with the dual-ViT image prefix."""

  def __init__(self, config: common.GriffinConfig,
               gradient_checkpointing: bool = True, device=None, dtype=None,
               vision: common.VisionConfig | None = None, compat: bool = True):
    super().__init__()
    self.config = config
    self.gradient_checkpointing = gradient_checkpointing  # inference: unused
    self.vision_config = vision
    self.compat = compat
    if vision is not None:
      self.vis_encoder = VisionEncoder(device=device, config=vision)
      self.projector = MLPProjector(device=device,
                                    hidden_depth=vision.projector_hidden_depth,
                                    in_features=vision.feature_width,
                                    width=config.width)
    self.embedder = modules.Embedder(config.vocab_size, config.width,
                                     config.embeddings_scale_by_sqrt_dim,
                                     device=device, dtype=dtype)
    self.blocks = nn.ModuleList([
        modules.ResidualBlock(
            width=config.width, mlp_expanded_width=config.mlp_expanded_width,
            num_heads=config.num_heads,
            attention_window_size=config.attention_window_size,
            temporal_block_type=kind, lru_width=config.lru_width,
            final_w_init_variance_scale=2.0 / config.num_layers,
            device=device, dtype=dtype, compat=compat)
        for kind in config.block_types
    ])
    self.final_norm = layers.RMSNorm(config.width, device=device, dtype=dtype)

  def reset_parameters(self) -> None:
    self.embedder.reset_parameters()
    for block in self.blocks:
      block.reset_parameters()
    self.final_norm.reset_parameters()

  # ------------------------------------------------------------- internals

  @property
  def n_visual_tokens(self) -> int:
    return 0 if self.vision_config is None else self.vision_config.n_visual_tokens

  def _pixels(self, images, img_path, batch: int):
    dev = self.embedder.input_embedding.device
    if images is not None:
      return images.to(dev, torch.float32).contiguous()
    from . import image_io
    px = image_io.load_images(img_path, self.vision_config.image_size, dev)
    if px.shape[0] == batch:        # a list of B paths: one image per sample
      return px
    if px.shape[0] != 1:
      raise ValueError(f"{px.shape[0]} images for a batch of {batch}")
    return px.expand(batch, -1, -1, -1).contiguous()   # reference: one image

  def embed_inputs(self, tokens, segment_pos, images=None, img_path=None,
                   image_splice=None):
    """Returns (x [B*L, D], positions [B, L] int32, L) with the image spliced.

    `image_splice` (host bool) is the caller's answer to griffin.py:179's
    "does the prompt hold a position 0" when it knows it without a device
    sync (the sampler computes positions on the host); None = check here."""
    b, t = tokens.shape
    d = self.config.width
    dev = tokens.device
    pos = segment_pos.to(torch.int32).contiguous()
    if (images is not None or img_path) and self.vision_config is None:
      raise ValueError("images / img_path were given to a Griffin built "
                       "without a vision tower (vision=None)")
    want_image = images is not None or bool(img_path)
    if want_image and image_splice is None:
      image_splice = bool((pos == 0).any())              # griffin.py:179
    if want_image and image_splice:
      n_vis = self.n_visual_tokens
      length = n_vis + t
      x = torch.empty(b * length, d, dtype=self.embedder.input_embedding.dtype,
                      device=dev)
      feats = torch.empty(b * n_vis, self.vision_config.feature_width,
                          dtype=torch.bfloat16, device=dev)
      with trace("vision_encoder"):
        self.vis_encoder.features_into(self._pixels(images, img_path, b), feats)
      with trace("projector"):
        self.projector.project_into(feats, x, row_map=(n_vis, length, 0))
      self.embedder.encode_into(tokens, x, row_map=(t, length, n_vis))
      pos = ops.ops.splice_positions(pos, n_vis)
      return x, pos, length
    x = torch.empty(b * t, d, dtype=self.embedder.input_embedding.dtype,
                    device=dev)
    self.embedder.encode_into(tokens, x)
    return x, pos, t

  def run_blocks(self, x, pos, b, length, cache, return_cache,
                 inplace_state=False, final_norm=False, xn0=None):
    """Runs the residual blocks; each block's last GEMM also produces the
    next norm's output (xn0: the first block's, e.g. the decode step's lazy
    PackedRows).  Returns (x, final_norm(x) if final_norm else None,
    cache)."""
    new_cache = {}
    xn = xn0
    n = len(self.blocks)
    for i, block in enumerate(self.blocks):
      name = f"blocks.{i}"
      nxt = (self.blocks[i + 1].temporal_pre_norm if i + 1 < n else
             (self.final_norm if final_norm else None))
      with trace(f"{name}:{block.temporal_block_type.name.lower()}"):
        x, xn, new_cache[name] = block.fused(
            x, pos, b, length, None if cache is None else cache[name],
            return_cache, inplace_state, xn, nxt, next_lazy=i + 1 < n)
    if final_norm and xn is None:
      xn = ops.rmsnorm(x, self.final_norm.scale, self.final_norm.eps,
                       packed=True)
    return x, xn, new_cache

  # ------------------------------------------------------------------ API

  @torch.no_grad()
  def forward(self, tokens: torch.Tensor, segment_pos: torch.Tensor,
              cache: Cache | None = None, return_logits: bool = True,
              return_cache: bool = True, img_path: str | list[str] | None = None,
              images: torch.Tensor | None = None, *,
              image_splice: bool | None = None):
    if not return_logits and not return_cache:
      return None, None
    if tokens.ndim == 1:
      tokens = tokens[None, :]
    if segment_pos.ndim == 1:
      segment_pos = segment_pos[None, :]
    b = tokens.shape[0]
    x, pos, length = self.embed_inputs(tokens, segment_pos, images, img_path,
                                       image_splice)
    x, xn, new_cache = self.run_blocks(x, pos, b, length, cache, return_cache,
                                       final_norm=return_logits)
    if not return_cache:
      new_cache = None
    if not return_logits:
      return None, new_cache
    logits = ops.gemm_logits(xn, self.embedder.input_embedding,
                             float(self.config.logits_soft_cap or 0.0))
    return logits.view(b, length, -1), new_cache

  @torch.no_grad()
  def next_token(self, tokens: torch.Tensor, segment_pos: torch.Tensor,
                 cache: Cache, return_logits: bool = False,
                 inplace: bool = True):
    """One decode step (T = 1) fused with soft-cap + greedy argmax.

    Recurrent and attention states are updated in place when `inplace`
    (what a captured hipGraph needs); returns (next [B] int32, logits
    [B, V] or None, cache).
    """
    b = tokens.shape[0]
    xn0 = None
    if ops.want_packed(b, self.config.width) and tokens.is_cuda:
      # one launch for the embedding in both layouts; the first block's
      # decode GEMVs apply its temporal_pre_norm on load, as every later
      # block's do (no separate RMSNorm launch)
      x, xn0 = self.embedder.encode_packed(tokens, self.blocks[0].temporal_pre_norm)
      pos = segment_pos.reshape(b, 1).to(torch.int32).contiguous()
    else:
      x, pos, _ = self.embed_inputs(tokens.reshape(b, 1),
                                    segment_pos.reshape(b, 1))
    x, xn, new_cache = self.run_blocks(x, pos, b, 1, cache, True, inplace,
                                       final_norm=True, xn0=xn0)
    logits, nxt = ops.logits_argmax(
        xn, self.embedder.input_embedding,
        float(self.config.logits_soft_cap or 0.0), return_logits)
    return nxt, (logits if return_logits else None), new_cache

  @torch.no_grad()
  def next_token_chained(self, x: torch.Tensor, xp: torch.Tensor,
                         segment_pos: torch.Tensor, cache: Cache, tail: dict):
    """One greedy decode step (T = 1, B <= 32) of a captured decode loop
    whose input rows come from the previous step: `x` [B, D] / `xp` (packed)
    hold the current token's embedding (Embedder.encode_packed), and the step
    ends in one tail launch (ops.logits_argmax_tail) that does the argmax,
    the decode_advance_ bookkeeping (tail: buf, step, pos, cur, done,
    eos_args, counter) and writes the NEXT token's embedding back into x /
    xp.  States update in place; returns next [B] int32."""
    b, d = x.shape
    pos = segment_pos.reshape(b, 1)
    xn0 = ops.PackedRows(xp, b, d, self.blocks[0].temporal_pre_norm, x)
    _, xn, _ = self.run_blocks(x, pos, b, 1, cache, True, True, final_norm=True,
                               xn0=xn0)
    return ops.logits_argmax_tail(
        xn, self.embedder.input_embedding,
        float(self.config.logits_soft_cap or 0.0),
        dict(tail, x=x, xp=xp, scale=self.embedder.scale))

  def init_cache(self, batch_size: int, dtype: torch.dtype) -> Cache:
    dev = self.embedder.input_embedding.device
    cfg = self.config
    return {
        f"blocks.{i}": modules.ResidualBlock.init_cache(
            batch_size=batch_size, width=cfg.width, num_heads=cfg.num_heads,
            attention_window_size=cfg.attention_window_size,
            temporal_block_type=kind, dtype=dtype, lru_width=cfg.lru_width,
            device=dev)
        for i, kind in enumerate(cfg.block_types)
    }
