"""Dual vision tower (DINOv2-L/14-reg4 + SigLIP-so400m/14) on MI355X.

Replaces `recurrentgemma/vit/dino_siglip.py` (`VisionEncoder` :19-156).  The
reference builds two timm `VisionTransformer`s and takes
`get_intermediate_layers(n={len(dino.blocks) - 2})` from both (block 22, no
final norm, prefix tokens dropped; :85-86), then concatenates the features
(:153-154).  Here each encoder keeps timm's parameter names (state-dict
compatible with a timm checkpoint) and runs as gfx950 kernels:

  im2col+Normalize -> patch GEMM (+bias +pos_embed, fp32 stream) -> prefix
  per block: LayerNorm -> qkv GEMM -> fused SDPA -> proj GEMM (+LayerScale
  +residual, fp32) -> LayerNorm -> fc1 GEMM (+GELU) -> fc2 GEMM (+LS +res)
  -> bf16 feature columns of the projector input.

The residual stream stays fp32 like the reference's fp32 timm model; GEMM
operands are bf16 with fp32 accumulation (tolerance: SURVEY §8c).
"""

from __future__ import annotations

import math

import torch
from torch import nn

from . import common, ops
from .layers import PackCache


def _pad_to(n: int, m: int) -> int:
  return (n + m - 1) // m * m


def _trunc_normal_(t: torch.Tensor, std: float):
  nn.init.trunc_normal_(t, mean=0.0, std=std, a=-2 * std, b=2 * std)


class LayerScale(nn.Module):
  def __init__(self, dim: int, init_values: float = 1e-5, device=None,
               dtype=None):
    super().__init__()
    self.gamma = nn.Parameter(init_values * torch.ones(dim, device=device,
                                                       dtype=dtype))


class Attention(nn.Module):
  def __init__(self, dim: int, num_heads: int, device=None, dtype=None):
    super().__init__()
    self.num_heads = num_heads
    self.qkv = nn.Linear(dim, 3 * dim, bias=True, device=device, dtype=dtype)
    self.proj = nn.Linear(dim, dim, bias=True, device=device, dtype=dtype)


class Mlp(nn.Module):
  def __init__(self, dim: int, hidden: int, device=None, dtype=None):
    super().__init__()
    self.fc1 = nn.Linear(dim, hidden, device=device, dtype=dtype)
    self.fc2 = nn.Linear(hidden, dim, device=device, dtype=dtype)


class Block(nn.Module):
  """timm `Block` parameter layout (norm1, attn, ls1, norm2, mlp, ls2)."""

  def __init__(self, cfg: common.ViTConfig, device=None, dtype=None):
    super().__init__()
    kw = dict(device=device, dtype=dtype)
    self.norm1 = nn.LayerNorm(cfg.width, eps=1e-6, **kw)
    self.attn = Attention(cfg.width, cfg.num_heads, **kw)
    self.norm2 = nn.LayerNorm(cfg.width, eps=1e-6, **kw)
    self.mlp = Mlp(cfg.width, cfg.mlp_width, **kw)
    if cfg.layer_scale:
      self.ls1 = LayerScale(cfg.width, **kw)
      self.ls2 = LayerScale(cfg.width, **kw)
    self._packed = PackCache()
    self.cfg = cfg

  def fc_packed(self):
    """fc1 rows / fc2 columns zero-padded to a multiple of 128 / 64."""
    def build():
      h = self.cfg.mlp_width
      hp = _pad_to(h, 128)
      d = self.cfg.width
      w1 = torch.zeros(hp, d, dtype=self.mlp.fc1.weight.dtype,
                       device=self.mlp.fc1.weight.device)
      w1[:h] = self.mlp.fc1.weight
      b1 = torch.zeros(hp, dtype=w1.dtype, device=w1.device)
      b1[:h] = self.mlp.fc1.bias
      w2 = torch.zeros(d, hp, dtype=w1.dtype, device=w1.device)
      w2[:, :h] = self.mlp.fc2.weight
      return w1, b1, w2
    return self._packed.get([self.mlp.fc1.weight, self.mlp.fc1.bias,
                             self.mlp.fc2.weight], build)

  def run(self, resid2d: torch.Tensor, b: int, ntok: int):
    cfg = self.cfg
    h = ops.ops.layernorm(resid2d, self.norm1.weight, self.norm1.bias, 1e-6)
    qkv = ops.linear(h, self.attn.qkv.weight, self.attn.qkv.bias)
    att = ops.ops.vit_attention(qkv, b, ntok, cfg.num_heads, cfg.head_dim)
    ops.ops.vit_residual_(att, self.attn.proj.weight, self.attn.proj.bias,
                          self.ls1.gamma if cfg.layer_scale else None, resid2d)
    h = ops.ops.layernorm(resid2d, self.norm2.weight, self.norm2.bias, 1e-6)
    w1, b1, w2 = self.fc_packed()
    f = ops.linear(h, w1, b1, act=3 if cfg.gelu_tanh else 1)
    ops.ops.vit_residual_(f, w2, self.mlp.fc2.bias,
                          self.ls2.gamma if cfg.layer_scale else None, resid2d)


class PatchEmbed(nn.Module):
  def __init__(self, cfg: common.ViTConfig, device=None, dtype=None):
    super().__init__()
    self.proj = nn.Conv2d(3, cfg.width, cfg.patch_size, cfg.patch_size,
                          bias=True, device=device, dtype=dtype)


class VisionTransformer(nn.Module):
  """One timm-style encoder, run up to `blocks_run` blocks."""

  def __init__(self, cfg: common.ViTConfig, image_size: int, device=None,
               dtype=None):
    super().__init__()
    self.cfg = cfg
    self.image_size = image_size
    g = image_size // cfg.patch_size
    self.num_patches = g * g
    kw = dict(device=device, dtype=dtype)
    self.patch_embed = PatchEmbed(cfg, **kw)
    if cfg.class_token:
      self.cls_token = nn.Parameter(torch.zeros(1, 1, cfg.width, **kw))
    if cfg.reg_tokens:
      self.reg_token = nn.Parameter(torch.zeros(1, cfg.reg_tokens, cfg.width,
                                                **kw))
    self.pos_embed = nn.Parameter(torch.zeros(1, self.num_patches, cfg.width,
                                              **kw))
    self.blocks = nn.ModuleList([Block(cfg, **kw) for _ in range(cfg.depth)])
    self.norm = nn.LayerNorm(cfg.width, eps=1e-6, **kw)   # unused (norm=False)
    self._packed = PackCache()
    self.reset_parameters()

  def reset_parameters(self) -> None:
    """timm-style init: trunc-normal 0.02 linears/pos, LayerScale 1e-5."""
    with torch.no_grad():
      _trunc_normal_(self.pos_embed, 0.02)
      if self.cfg.class_token:
        nn.init.normal_(self.cls_token, std=1e-6)
      if self.cfg.reg_tokens:
        nn.init.normal_(self.reg_token, std=1e-6)
      fan_in = 3 * self.cfg.patch_size ** 2
      nn.init.uniform_(self.patch_embed.proj.weight, -1 / math.sqrt(fan_in),
                       1 / math.sqrt(fan_in))
      nn.init.zeros_(self.patch_embed.proj.bias)
      for blk in self.blocks:
        for lin in (blk.attn.qkv, blk.attn.proj, blk.mlp.fc1, blk.mlp.fc2):
          _trunc_normal_(lin.weight, 0.02)
          nn.init.zeros_(lin.bias)

  def patch_packed(self):
    def build():
      w = self.patch_embed.proj.weight
      k = w[0].numel()
      kp = _pad_to(k, 64)
      wp = torch.zeros(w.shape[0], kp, dtype=w.dtype, device=w.device)
      wp[:, :k] = w.reshape(w.shape[0], k)
      pre = []
      if self.cfg.class_token:
        pre.append(self.cls_token.reshape(1, -1))
      if self.cfg.reg_tokens:
        pre.append(self.reg_token.reshape(self.cfg.reg_tokens, -1))
      prefix = torch.cat(pre).contiguous() if pre else None
      return wp, prefix, self.pos_embed.reshape(self.num_patches, -1).contiguous()
    src = [self.patch_embed.proj.weight, self.pos_embed]
    if self.cfg.class_token:
      src.append(self.cls_token)
    if self.cfg.reg_tokens:
      src.append(self.reg_token)
    return self._packed.get(src, build)

  def features_into(self, pixels: torch.Tensor, out2d: torch.Tensor,
                    col_off: int, blocks_run: int):
    """Runs the encoder on [B,3,S,S] pixels in [0,1]; writes bf16 features of
    block `blocks_run - 1` (prefix dropped) to out2d[:, col_off:col_off+D]."""
    for _ in self.feature_steps(pixels, out2d, col_off, blocks_run):
      pass

  def feature_steps(self, pixels: torch.Tensor, out2d: torch.Tensor,
                    col_off: int, blocks_run: int):
    """features_into as a generator: one yield after each enqueued block, so
    a caller can interleave the launches of two encoders on two streams."""
    cfg = self.cfg
    b = pixels.shape[0]
    assert pixels.shape[-1] == self.image_size, "image size mismatch"
    wp, prefix_tok, pos = self.patch_packed()
    patches = ops.ops.im2col_normalize(pixels, list(cfg.mean), list(cfg.std),
                                       cfg.patch_size, wp.shape[1])
    npre = cfg.num_prefix_tokens
    ntok = self.num_patches + npre
    resid = torch.empty(b, ntok, cfg.width, dtype=torch.float32,
                        device=pixels.device)
    ops.ops.patch_embed_(patches, wp, self.patch_embed.proj.bias, pos, resid,
                         b, self.num_patches, ntok, npre)
    if npre:
      ops.ops.vit_prefix_(prefix_tok, resid, b, ntok, npre)
    r2 = resid.view(b * ntok, cfg.width)
    for i in range(blocks_run):
      self.blocks[i].run(r2, b, ntok)
      yield i
    ops.ops.vit_features_(resid, out2d, col_off, b, ntok, npre)


class VisionEncoder(nn.Module):
  """Combined DINOv2 + SigLIP encoder (reference dino_siglip.py:19-156)."""

  def __init__(self, is_training: bool = False, device="cuda",
               default_image_size: int = 384,
               config: common.VisionConfig | None = None, dtype=torch.bfloat16):
    super().__init__()
    if config is None:
      config = common.VisionConfig(image_size=default_image_size)
    self.config = config
    self.is_training = is_training
    self.device = device
    self.default_image_size = config.image_size
    self.dino = VisionTransformer(config.dino, config.image_size, device, dtype)
    self.siglip = VisionTransformer(config.siglip, config.image_size, device,
                                    dtype)

  @property
  def n_visual_tokens(self) -> int:
    return self.config.n_visual_tokens

  def _side_stream(self, dev: torch.device) -> torch.cuda.Stream:
    """The SigLIP stream paired with the caller's current stream (callers on
    two streams -- pipelined micro-batches -- each get their own)."""
    sides = self.__dict__.setdefault("_sides", {})
    key = (dev, torch.cuda.current_stream(dev).cuda_stream)
    s = sides.get(key)
    if s is None:
      s = sides[key] = torch.cuda.Stream(device=dev)
    return s

  def features_into(self, pixels: torch.Tensor, out2d: torch.Tensor):
    """pixels [B,3,S,S] fp32 in [0,1] -> out2d [B*n_vis, 2176] bf16.

    The two encoders are independent until their feature columns meet in
    `out2d`, so SigLIP runs on a side stream beside DINO: the two towers'
    GEMMs (132-160 output tiles each at bs=32, 224 px) fill the 256 CUs
    together where either alone leaves ~40 % of them idle.  Not while a
    graph is being captured (one stream there), nor with `two_streams` set
    False on the encoder."""
    n = self.config.blocks_run
    if (torch.cuda.is_current_stream_capturing() or not pixels.is_cuda or
        not self.__dict__.get("two_streams", True)):
      self.dino.features_into(pixels, out2d, 0, n)
      self.siglip.features_into(pixels, out2d, self.config.dino.width, n)
      return
    cur = torch.cuda.current_stream(pixels.device)
    side = self._side_stream(pixels.device)
    side.wait_stream(cur)
    # the two towers' launches are interleaved block by block, so both
    # streams have work queued from the start (enqueueing one whole tower
    # first leaves the other stream idle for the host time that takes)
    dino = self.dino.feature_steps(pixels, out2d, 0, n)
    sig = self.siglip.feature_steps(pixels, out2d, self.config.dino.width, n)
    with ops.TIMER.scoped(" [vit, 2 streams]"):
      live = [True, True]
      while any(live):
        if live[1]:
          with torch.cuda.stream(side):
            live[1] = next(sig, None) is not None
        if live[0]:
          live[0] = next(dino, None) is not None
      pixels.record_stream(side)
      out2d.record_stream(side)
    cur.wait_stream(side)

  def encode(self, pixels: torch.Tensor) -> torch.Tensor:
    b = pixels.shape[0]
    out = torch.empty(b * self.n_visual_tokens, self.config.feature_width,
                      dtype=torch.bfloat16, device=pixels.device)
    self.features_into(pixels.contiguous(), out)
    return out.view(b, self.n_visual_tokens, -1)

  def forward(self, img_path_or_pixels) -> torch.Tensor:
    """`forward(img_path)` (reference API), a list of paths (one image per
    sample, resized on the GPU), or `forward(pixels [B,3,S,S])`."""
    if isinstance(img_path_or_pixels, (str, list, tuple)):
      from . import image_io
      pixels = image_io.load_images(img_path_or_pixels, self.config.image_size,
                                    self.device)
    else:
      pixels = img_path_or_pixels
    return self.encode(pixels)


class MLPProjector(nn.Module):
  """Linear(2176->2560) GELU [Linear(2560->2560) GELU]* Linear(2560->2560),
  bf16 (reference projector/mlp.py:7-31; keys proj.0/2/4)."""

  def __init__(self, device="cuda", hidden_depth: int = 2, in_features: int = 2176,
               width: int = 2560):
    super().__init__()
    self.device = device
    self.hidden_depth = hidden_depth
    layers: list[nn.Module] = [nn.Linear(in_features, width, device=device,
                                         dtype=torch.bfloat16), nn.GELU()]
    for _ in range(hidden_depth - 1):
      layers += [nn.Linear(width, width, device=device, dtype=torch.bfloat16),
                 nn.GELU()]
    layers.append(nn.Linear(width, width, device=device, dtype=torch.bfloat16))
    self.proj = nn.Sequential(*layers)

  def linears(self) -> list[nn.Linear]:
    return [m for m in self.proj if isinstance(m, nn.Linear)]

  def project_into(self, feats2d: torch.Tensor, out2d: torch.Tensor,
                   row_map=None):
    lins = self.linears()
    x = feats2d
    for lin in lins[:-1]:
      x = ops.linear(x, lin.weight, lin.bias, act=1)
    ops.linear(x, lins[-1].weight, lins[-1].bias, out=out2d, row_map=row_map)

  def forward(self, x: torch.Tensor) -> torch.Tensor:
    shape = x.shape
    x2 = x.reshape(-1, shape[-1]).to(torch.bfloat16).contiguous()
    out = torch.empty(x2.shape[0], self.linears()[-1].out_features,
                      dtype=torch.bfloat16, device=x.device)
    self.project_into(x2, out)
    return out.view(*shape[:-1], -1)
