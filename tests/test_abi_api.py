"""C-ABI library + Python API surface (CPU only; no compute calls)."""

import ctypes
import os
import re

import pytest
import torch

import cadence
from cadence import _lib, common, ops

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "cadence_kernels.h")


def declared_symbols():
  text = open(HEADER).read()
  text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
  return sorted(set(re.findall(r"\b(cadence_\w+)\s*\(", text)))


def test_library_loads_and_exports_every_declared_symbol():
  lib = _lib.load()
  syms = declared_symbols()
  assert len(syms) >= 25
  for s in syms:
    assert hasattr(lib, s), s
  assert set(syms) == set(_lib.exported_symbols())
  assert lib.cadence_abi_version() == _lib.ABI_VERSION


def test_copy_batched_contract_without_gpu():
  lib = _lib.load()
  assert lib.cadence_copy_batched(None, 0, None) == 0          # nothing to do
  bad = (_lib.CopyDesc * 1)(_lib.CopyDesc(16, 32, 1, 6, 0, 0))   # 6-byte rows
  assert lib.cadence_copy_batched(bad, 1, None) != 0
  bad = (_lib.CopyDesc * 1)(_lib.CopyDesc(18, 32, 1, 8, 0, 0))   # misaligned src
  assert lib.cadence_copy_batched(bad, 1, None) != 0
  bad = (_lib.CopyDesc * 1)(_lib.CopyDesc(16, 32, 2, 64, 32, 64))  # stride < row
  assert lib.cadence_copy_batched(bad, 1, None) != 0
  empty = (_lib.CopyDesc * 1)(_lib.CopyDesc(None, None, 0, 0, 0, 0))
  assert lib.cadence_copy_batched(empty, 1, None) == 0


def test_host_contract_checks_without_gpu():
  lib = _lib.load()
  # workspace query is host-only arithmetic
  assert lib.cadence_gemm_workspace_bytes(4096, 2560, 2560, 1) == 0
  assert lib.cadence_gemm_workspace_bytes(32, 2560, 7680, 1) > 0   # split K
  # contract violations are rejected before any launch (N % 64 != 0)
  assert lib.cadence_gemm_linear(None, 0, None, 0, None, None, 0, None, 0, 8,
                                 100, 64, 0, 8, 0, 0, None, 0, None) != 0


def test_decode_step_entry_points_reject_bad_shapes_without_gpu():
  """cadence_embed_packed / cadence_logits_argmax_tail (ABI 17) check their
  contract on the host before any launch."""
  lib = _lib.load()
  # 33 rows (> 32), D not a multiple of 32, no packed buffer
  assert lib.cadence_embed_packed(None, None, None, 2560, 8, 33, 2560, 256000, 1.0, None) != 0
  assert lib.cadence_embed_packed(None, None, None, 2568, 8, 32, 2568, 256000, 1.0, None) != 0
  assert lib.cadence_embed_packed(None, None, None, 2560, None, 32, 2560, 256000, 1.0,
                                  None) != 0
  assert lib.cadence_embed_packed(None, None, None, 2560, 8, 0, 2560, 256000, 1.0, None) == 0
  # no descriptor, no next-token buffer, 33 rows
  assert lib.cadence_logits_argmax_tail(None, 0, None, 0, 32, 256000, 2560, 30.0, 8, None, 0,
                                        None, None) != 0
  t = _lib.DecodeTail()
  assert lib.cadence_logits_argmax_tail(None, 0, None, 0, 33, 256000, 2560, 30.0, 8, None, 0,
                                        ctypes.byref(t), None) != 0
  # a descriptor without its counter / rows
  assert lib.cadence_logits_argmax_tail(None, 0, None, 0, 32, 256000, 2560, 30.0, 8, None, 0,
                                        ctypes.byref(t), None) != 0
  assert lib.cadence_logits_argmax_tail(None, 0, None, 0, 0, 256000, 2560, 30.0, None, None,
                                        0, None, None) == 0


def test_reference_exports_present():
  # recurrentgemma/torch/__init__.py:42-59
  for name in ("ScanType", "TemporalBlockType", "rnn_scan",
               "BlockDiagonalLinear", "RGLRU", "Conv1D", "RecurrentBlockCache",
               "RecurrentBlock", "AttentionBlockCache", "LocalAttentionBlock",
               "ResidualBlockCache", "ResidualBlock", "Preset",
               "GriffinConfig", "Griffin", "Sampler"):
    assert name in cadence.__all__ and hasattr(cadence, name), name
  assert hasattr(cadence, "VisionEncoder") and hasattr(cadence, "MLPProjector")


def test_preset_2b():
  cfg = common.GriffinConfig.from_preset(common.Preset.RECURRENT_GEMMA_2B_V1)
  assert (cfg.width, cfg.mlp_expanded_width, cfg.num_heads, cfg.lru_width,
          cfg.num_layers, cfg.attention_window_size,
          cfg.logits_soft_cap) == (2560, 7680, 10, 2560, 26, 2048, 30.0)
  kinds = [k.name[0] for k in cfg.block_types]
  assert "".join(kinds[:6]) == "RRARRA" and kinds.count("A") == 8
  assert common.GriffinConfig.from_preset(
      common.Preset.RECURRENT_GEMMA_2B_V1,
      max_sequence_length=512).attention_window_size == 512


def test_state_dict_keys_and_config_inference_cpu_init():
  RA = common.TemporalBlockType
  cfg = common.GriffinConfig(
      vocab_size=64, width=256, mlp_expanded_width=768, num_heads=4,
      block_types=(RA.RECURRENT, RA.ATTENTION),
      embeddings_scale_by_sqrt_dim=True, attention_window_size=64,
      logits_soft_cap=30.0)
  vis = common.VisionConfig(
      image_size=28,
      dino=common.ViTConfig("dino", 128, 1, 2, 256, class_token=True,
                            reg_tokens=4, layer_scale=True),
      siglip=common.ViTConfig("siglip", 128, 1, 2, 200),
      feature_block=0)
  m = cadence.Griffin(cfg, dtype=torch.bfloat16, vision=vis)
  sd = m.state_dict()
  expected = {
      "embedder.input_embedding", "final_norm.scale",
      "blocks.0.temporal_pre_norm.scale", "blocks.0.channel_pre_norm.scale",
      "blocks.0.recurrent_block.linear_x.weight",
      "blocks.0.recurrent_block.linear_y.bias",
      "blocks.0.recurrent_block.linear_out.weight",
      "blocks.0.recurrent_block.conv_1d.w", "blocks.0.recurrent_block.conv_1d.b",
      "blocks.0.recurrent_block.rg_lru.a_param",
      "blocks.0.recurrent_block.rg_lru.input_gate.w",
      "blocks.0.recurrent_block.rg_lru.a_gate.b",
      "blocks.0.mlp_block.ffw_up.w", "blocks.0.mlp_block.ffw_up.b",
      "blocks.0.mlp_block.ffw_down.weight", "blocks.0.mlp_block.ffw_down.bias",
      "blocks.1.attention_block.proj_q.weight",
      "blocks.1.attention_block.proj_k.weight",
      "blocks.1.attention_block.proj_v.weight",
      "blocks.1.attention_block.proj_final.weight",
      "blocks.1.attention_block.proj_final.bias",
      "projector.proj.0.weight", "projector.proj.2.bias",
      "projector.proj.4.weight",
      "vis_encoder.dino.patch_embed.proj.weight", "vis_encoder.dino.pos_embed",
      "vis_encoder.dino.cls_token", "vis_encoder.dino.reg_token",
      "vis_encoder.dino.blocks.0.norm1.weight",
      "vis_encoder.dino.blocks.0.attn.qkv.weight",
      "vis_encoder.dino.blocks.0.ls1.gamma",
      "vis_encoder.dino.blocks.0.mlp.fc2.bias",
      "vis_encoder.siglip.blocks.0.attn.proj.weight",
  }
  missing = expected - set(sd)
  assert not missing, missing
  assert sd["blocks.0.recurrent_block.rg_lru.a_gate.w"].shape == (4, 64, 64)
  assert sd["blocks.1.attention_block.proj_k.weight"].shape == (64, 256)
  assert sd["blocks.0.mlp_block.ffw_up.b"].shape == (2, 1, 1, 768)
  re_cfg = common.GriffinConfig.from_torch_params(
      sd, embeddings_scale_by_sqrt_dim=True, attention_window_size=64,
      logits_soft_cap=30.0)
  assert re_cfg.block_types == cfg.block_types
  assert re_cfg.num_heads == 4 and re_cfg.lru_width == 256
  with pytest.raises(ValueError):
    common.GriffinConfig.from_torch_params(
        sd, preset=common.Preset.RECURRENT_GEMMA_2B_V1)


def test_rg_lru_init_ring():
  """rnn_param_init: a = exp(-softplus(param)) lies in [0.9, 0.999]."""
  lru = cadence.RGLRU(512, 4)
  a = torch.exp(-torch.nn.functional.softplus(lru.a_param.detach()))
  assert a.min() >= 0.9 - 1e-4 and a.max() <= 0.999 + 1e-4


def test_ops_have_no_cpu_fallback():
  x = torch.zeros(4, 8, dtype=torch.bfloat16)
  with pytest.raises((NotImplementedError, RuntimeError)):
    torch.ops.cadence.rmsnorm(x, torch.zeros(8, dtype=torch.bfloat16), 1e-6)


def test_packed_rows_layout_matches_header_formula():
  """ops.pack_rows == the index formula of cadence_kernels.h ("Decode
  activation layout"), for full and partial 16-row tiles."""
  from cadence import ops
  for m, k in ((32, 64), (17, 96), (5, 32)):
    x = torch.arange(m * k, dtype=torch.float32).view(m, k).to(torch.bfloat16)
    p = ops.pack_rows(x)
    mt = -(-m // 16)
    assert p.data.numel() == k * 16 * mt
    for mm in range(m):
      for kk in range(k):
        idx = (((kk // 32) * mt + mm // 16) * 512 + (mm % 16 + 16 * ((kk % 32) // 8)) * 8
               + kk % 8)
        assert p.data[idx] == x[mm, kk], (m, k, mm, kk)
    assert torch.equal(p.unpack(), x)


def test_positions_and_sampler_prompt_layout():
  from cadence.sampler import prompt_positions
  pos = prompt_positions(torch.tensor([3, 5]), 5)
  assert pos.tolist() == [[-1, -1, 0, 1, 2], [0, 1, 2, 3, 4]]


def test_decode_tail_descriptor_layout():
  """cadence._lib.DecodeTail mirrors CadenceDecodeTail (the C side
  static_asserts the same size and offsets)."""
  import ctypes
  T = _lib.DecodeTail
  assert ctypes.sizeof(T) == 120
  assert T.counter.offset == 64 and T.scale.offset == 88 and T.packed_out.offset == 112


def test_prefill_gemm_plan_host_arithmetic():
  """The prefill engine's tile height and K-split plan (host-only; 256 CUs
  assumed when no GPU is visible): bench shapes keep one pass with the tile
  heights DESIGN §4 names, one-image / one-prompt shapes split K."""
  lib = _lib.load()
  rows = lib.cadence_gemm_tile_rows
  assert rows(32 * 319, 15360, 2560, 1) == 256        # Griffin gated MLP (4-wave engine)
  assert rows(32 * 2048, 15360, 2560, 1) == 224       # C2's gated MLP (4-wave engine)
  assert rows(32 * 319, 2560, 7680, 1) == 224         # Griffin down projection
  assert rows(32 * 261, 1024, 1024, 1) == 160         # DINO attention proj
  assert rows(32 * 256, 1152, 1152, 1) == 192         # SigLIP attention proj
  assert rows(32 * 261, 4096, 1024, 1) == 192         # DINO fc1
  splits = lib.cadence_gemm_big_splits
  assert splits(32 * 319, 15360, 2560, 1) == 1
  assert splits(32 * 261, 1024, 1024, 1) == 1
  assert splits(261, 3072, 1024, 1) == 4               # C3 ViT qkv: K 1024
  assert splits(319, 2560, 7680, 1) == 6               # C3 down projection
  assert splits(319, 15360, 2560, 1) == 2              # C3 gated MLP
  assert splits(319, 2560, 2560, 8) == 1               # grouped launches never split
  s = splits(319, 2560, 7680, 1)
  assert lib.cadence_gemm_workspace_bytes(319, 2560, 7680, 1) == s * 319 * 2560 * 4


def test_roctx_ranges_nest():
  """SURVEY §5 tracing: the roctx ranges are opt-in and nest (push / pop)."""
  from cadence import tracing
  prev = tracing.enabled()
  tracing.enable(True)
  try:
    with tracing.trace("outer"):
      with tracing.trace("inner"):
        pass
  finally:
    tracing.enable(prev)
  assert tracing.enabled() == prev



def test_rglru_gates_plan_query():
  """cadence_rglru_gates_stream_plan (host-only): the streaming gates kernel
  for aligned row-major prefill operands of a width it has, the block engine
  otherwise (packed decode weights, M <= 32, other widths, odd strides,
  misaligned rows, or the lab switch's engine bit 1 clear)."""
  lib = _lib.load()
  plan = lib.cadence_rglru_gates_stream_plan
  A, W = 0x10000, 0x20000
  assert plan(A, 5120, W, 256, 2560, 10208, 256) == 1
  assert plan(A, 512, W, 64, 512, 100, 64) == 1
  assert plan(A, 5120, W, 0, 2560, 10208, 256) == 0      # fragment-packed
  assert plan(A, 5120, W, 256, 2560, 32, 256) == 0       # decode rows
  assert plan(A, 5120, W, 192, 2560, 10208, 192) == 0    # no instance
  assert plan(A + 2, 5120, W, 256, 2560, 10208, 256) == 0
  assert plan(A, 5121, W, 256, 2560, 10208, 256) == 0
  prev = lib.cadence_gemm_set_engine(0)
  try:
    assert plan(A, 5120, W, 256, 2560, 10208, 256) == 0
  finally:
    lib.cadence_gemm_set_engine(prev)


def test_vit_attention_plan_query():
  """cadence_vit_attention_kernel (host-only): DINO's 224-px shape on the
  LDS-resident kernel, every other tower shape on vit_flash_attn_kernel, the
  round-3 kernels with the lab switch's bit 3 clear."""
  lib = _lib.load()
  plan = lib.cadence_vit_attention_kernel
  assert plan(261, 64) == 0
  assert [plan(n, hd) for n, hd in ((256, 72), (581, 64), (576, 72), (734, 64), (729, 72))] \
      == [2] * 5
  assert plan(100, 80) == -1
  prev = lib.cadence_gemm_set_engine(-1)
  lib.cadence_gemm_set_engine(prev & ~8)
  try:
    assert (plan(256, 72), plan(581, 64)) == (0, 1)
  finally:
    lib.cadence_gemm_set_engine(prev)


def test_recurrent_decode_front_plan_query():
  """cadence_recurrent_decode_front_plan (host-only): the one-launch decode
  recurrent front takes 17..32 rows, gate blocks of 64..256 channels that
  tile the width, and a K that the weight-streaming engine covers in one
  split of ten 32-deep k-steps per wave; the host mirror leaves it off by
  default (measured slower than the two launches)."""
  lib = _lib.load()
  plan = lib.cadence_recurrent_decode_front_plan
  assert plan(32, 2560, 2560, 10, 256) == 1            # CadenceGemma-2B, bench batch
  assert plan(17, 2560, 2560, 10, 256) == 1
  assert plan(24, 1024, 1280, 8, 128) == 1
  assert plan(16, 2560, 2560, 10, 256) == 0            # one 16-row tile
  assert plan(33, 2560, 2560, 10, 256) == 0            # not decode rows
  assert plan(32, 2560, 2560, 10, 192) == 0            # block width
  assert plan(32, 2560, 2560, 9, 256) == 0             # heads x bw != E
  assert plan(32, 2560, 1024, 10, 256) == 0            # K below the 10-step plan
  assert plan(32, 2560, 7680, 10, 256) == 0            # K needs a split
  assert plan(32, 5120, 2560, 20, 256) == 0            # > 256 workgroups
  assert ops.FRONT_ONE_LAUNCH is False
