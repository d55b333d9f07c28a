"""Model configuration shared by the host path and the tests.

Restates the public configuration API of the reference
(`recurrentgemma/common.py`): `TemporalBlockType` (:22-27), `ScanType`
(:30-42), `Preset` (:45-114), `GriffinConfig` (:117-410) and
`apply_it_formatter` (:413-414).  Field names, defaults and error behaviour
are kept so that reference call sites (`GriffinConfig.from_preset`,
`GriffinConfig.from_torch_params(...)`) work unchanged.

Added for the multimodal path: `VisionConfig` (the dual DINOv2/SigLIP tower
of `recurrentgemma/vit/dino_siglip.py:57-130`) and `n_visual_tokens`, which
generalises the hard-coded 729 of `recurrentgemma/torch/griffin.py:188`
(SURVEY Appendix A, Q2).
"""

from __future__ import annotations

import dataclasses
import enum
import itertools
from typing import Any, Mapping, NamedTuple


@enum.unique
class TemporalBlockType(enum.Enum):
  """Temporal-mixing sub-block of a residual block."""

  ATTENTION = enum.auto()
  RECURRENT = enum.auto()


@enum.unique
class ScanType(enum.Enum):
  """Kept for API compatibility (the reference uses it for its JAX scan).

  On MI355X every value maps to the same HIP linear-recurrence kernel.
  """

  AUTO = enum.auto()
  LINEAR_NATIVE = enum.auto()
  ASSOCIATIVE_NATIVE = enum.auto()
  LINEAR_PALLAS = enum.auto()


def _griffin_pattern(n: int) -> tuple[TemporalBlockType, ...]:
  cyc = itertools.cycle((TemporalBlockType.RECURRENT,
                         TemporalBlockType.RECURRENT,
                         TemporalBlockType.ATTENTION))
  return tuple(itertools.islice(cyc, n))


@enum.unique
class Preset(enum.Enum):
  """Preset architectures (values from `recurrentgemma/common.py:62-114`)."""

  GRIFFIN_PAPER_7B = enum.auto()
  HAWK_PAPER_7B = enum.auto()
  RECURRENT_GEMMA_2B_V1 = enum.auto()
  RECURRENT_GEMMA_9B_V1 = enum.auto()

  @property
  def config_dict(self) -> dict[str, Any]:
    table = {
        Preset.GRIFFIN_PAPER_7B: dict(
            width=4096, mlp_expanded_width=3 * 4096, num_heads=32,
            lru_width=5632, block_types=_griffin_pattern(32),
            embeddings_scale_by_sqrt_dim=False, attention_window_size=1024,
            logits_soft_cap=0.0, scan_type=ScanType.AUTO),
        Preset.HAWK_PAPER_7B: dict(
            width=4096, mlp_expanded_width=3 * 4096, num_heads=32,
            lru_width=5632, block_types=(TemporalBlockType.RECURRENT,) * 32,
            embeddings_scale_by_sqrt_dim=False, attention_window_size=1024,
            logits_soft_cap=0.0, scan_type=ScanType.AUTO),
        Preset.RECURRENT_GEMMA_2B_V1: dict(
            width=2560, mlp_expanded_width=3 * 2560, num_heads=10,
            lru_width=2560, block_types=_griffin_pattern(26),
            embeddings_scale_by_sqrt_dim=True, attention_window_size=2048,
            logits_soft_cap=30.0, scan_type=ScanType.AUTO),
        Preset.RECURRENT_GEMMA_9B_V1: dict(
            width=4096, mlp_expanded_width=3 * 4096, num_heads=16,
            lru_width=4096, block_types=_griffin_pattern(38),
            embeddings_scale_by_sqrt_dim=True, attention_window_size=2048,
            logits_soft_cap=30.0, scan_type=ScanType.AUTO),
    }
    return dict(table[self])


class GriffinConfig(NamedTuple):
  """Griffin language-model hyper-parameters (reference `common.py:117-152`)."""

  vocab_size: int
  width: int
  mlp_expanded_width: int
  num_heads: int
  block_types: tuple[TemporalBlockType, ...]
  embeddings_scale_by_sqrt_dim: bool
  attention_window_size: int
  logits_soft_cap: float
  lru_width: int | None = None
  scan_type: ScanType = ScanType.AUTO

  @property
  def max_cache_length(self) -> int:
    return self.attention_window_size

  @property
  def num_layers(self) -> int:
    return len(self.block_types)

  @property
  def head_dim(self) -> int:
    return self.width // self.num_heads

  @property
  def rnn_width(self) -> int:
    return self.lru_width or self.width

  @classmethod
  def from_preset(cls, preset: Preset, vocab_size: int = 256_000,
                  max_sequence_length: int | None = None) -> "GriffinConfig":
    kw = preset.config_dict
    if max_sequence_length is not None:
      kw["attention_window_size"] = min(kw["attention_window_size"],
                                        max_sequence_length)
    return cls(vocab_size=vocab_size, **kw)

  @classmethod
  def _from_parameter_kwargs(cls, kwargs, preset=None,
                             embeddings_scale_by_sqrt_dim=None,
                             attention_window_size=None,
                             logits_soft_cap=None,
                             scan_type=ScanType.AUTO,
                             max_sequence_length=None):
    # Same validation contract as reference common.py:179-220.
    defaults: dict[str, Any] = {}
    if preset is not None:
      defaults = preset.config_dict
      for key, value in kwargs.items():
        if key != "vocab_size" and value != defaults[key]:
          raise ValueError(
              "The parameters provided does not seem to match the preset "
              f"{preset} provided, because the value for {key} is {value}, "
              f"which is not equal to the preset value of {defaults[key]}.")
    merged = dict(kwargs)
    for key, value in dict(
        embeddings_scale_by_sqrt_dim=embeddings_scale_by_sqrt_dim,
        attention_window_size=attention_window_size,
        logits_soft_cap=logits_soft_cap,
        scan_type=scan_type).items():
      merged[key] = value if value is not None else defaults.get(key)
    if max_sequence_length is not None:
      merged["attention_window_size"] = min(merged["attention_window_size"],
                                            max_sequence_length)
    return cls(**merged)

  @classmethod
  def from_torch_params(cls, params: Mapping[str, Any],
                        preset: Preset | None = None,
                        embeddings_scale_by_sqrt_dim: bool | None = None,
                        attention_window_size: int | None = None,
                        logits_soft_cap: float | None = None,
                        scan_type: ScanType | None = None,
                        max_sequence_length: int | None = None
                        ) -> "GriffinConfig":
    """Infers the architecture from a torch state dict (ref :323-410)."""
    vocab_size, width = params["embedder.input_embedding"].shape
    mlp_width = params["blocks.0.mlp_block.ffw_up.w"].shape[-1]
    lru_width = None
    num_heads = None
    kinds = []
    i = 0
    while f"blocks.{i}.channel_pre_norm.scale" in params:
      gate = f"blocks.{i}.recurrent_block.rg_lru.a_gate.w"
      proj_k = f"blocks.{i}.attention_block.proj_k.weight"
      if gate in params:
        kinds.append(TemporalBlockType.RECURRENT)
        nh, hd, _ = params[gate].shape
        num_heads, lru_width = nh, nh * hd
      elif proj_k in params:
        kinds.append(TemporalBlockType.ATTENTION)
        num_heads = width // params[proj_k].shape[0]
      else:
        raise ValueError(f"Can't recongnize the type of blocks.{i}.")
      i += 1
    return cls._from_parameter_kwargs(
        kwargs=dict(vocab_size=vocab_size, width=width,
                    mlp_expanded_width=mlp_width, num_heads=num_heads,
                    lru_width=lru_width, block_types=tuple(kinds)),
        preset=preset,
        embeddings_scale_by_sqrt_dim=embeddings_scale_by_sqrt_dim,
        attention_window_size=attention_window_size,
        logits_soft_cap=logits_soft_cap,
        scan_type=scan_type if scan_type is not None else ScanType.AUTO,
        max_sequence_length=max_sequence_length)


def apply_it_formatter(input_string: str) -> str:
  """Instruction-tuned prompt wrapper (reference `common.py:413-414`)."""
  return ("<start_of_turn>user\n" + input_string + "<end_of_turn>\n"
          "<start_of_turn>model\n")


# ----------------------------------------------------------------------------
# Vision tower (recurrentgemma/vit/dino_siglip.py:57-130).
# ----------------------------------------------------------------------------

IMAGENET_MEAN = (0.485, 0.456, 0.406)
IMAGENET_STD = (0.229, 0.224, 0.225)
SIGLIP_MEAN = (0.5, 0.5, 0.5)
SIGLIP_STD = (0.5, 0.5, 0.5)


@dataclasses.dataclass(frozen=True)
class ViTConfig:
  """One timm-style `VisionTransformer` encoder, as used by the reference.

  Attributes mirror the timm model arguments the reference instantiates
  (`vit_large_patch14_reg4_dinov2.lvd142m`, `vit_so400m_patch14_siglip_384`).
  """

  name: str
  width: int
  depth: int
  num_heads: int
  mlp_width: int
  patch_size: int = 14
  class_token: bool = False
  reg_tokens: int = 0
  layer_scale: bool = False
  gelu_tanh: bool = False
  mean: tuple[float, float, float] = IMAGENET_MEAN
  std: tuple[float, float, float] = IMAGENET_STD

  @property
  def head_dim(self) -> int:
    return self.width // self.num_heads

  @property
  def num_prefix_tokens(self) -> int:
    return int(self.class_token) + self.reg_tokens


DINOV2_L14_REG4 = ViTConfig(
    name="dino", width=1024, depth=24, num_heads=16, mlp_width=4096,
    class_token=True, reg_tokens=4, layer_scale=True,
    mean=IMAGENET_MEAN, std=IMAGENET_STD)

# timm default activation for the SigLIP ViT is erf-GELU (nn.GELU); the
# original big_vision model uses tanh-GELU.  Knob: `gelu_tanh`.
SIGLIP_SO400M_P14 = ViTConfig(
    name="siglip", width=1152, depth=27, num_heads=16, mlp_width=4304,
    class_token=False, reg_tokens=0, layer_scale=False,
    mean=SIGLIP_MEAN, std=SIGLIP_STD)


@dataclasses.dataclass(frozen=True)
class VisionConfig:
  """The dual vision tower of `dino_siglip.py` + the projector of `mlp.py`."""

  image_size: int = 384
  dino: ViTConfig = DINOV2_L14_REG4
  siglip: ViTConfig = SIGLIP_SO400M_P14
  # `get_intermediate_layers(n={len(dino.blocks) - 2})` for BOTH encoders
  # (dino_siglip.py:85-86): block index 22 -> 23 blocks are run (Q12).
  feature_block: int = 22
  projector_width: int = 2560
  projector_hidden_depth: int = 2

  @property
  def grid(self) -> int:
    return self.image_size // self.dino.patch_size

  @property
  def n_visual_tokens(self) -> int:
    return self.grid * self.grid

  @property
  def feature_width(self) -> int:
    return self.dino.width + self.siglip.width

  @property
  def blocks_run(self) -> int:
    return self.feature_block + 1
