"""cadence -- MI355X-native CadenceGemma multimodal forward path.

Drop-in for the `recurrentgemma.torch` public API (reference
`recurrentgemma/torch/__init__.py:24-59`) plus the vision tower and
projector of `recurrentgemma/vit` and `recurrentgemma/projector`:

    from cadence import GriffinConfig, Preset, Griffin, Sampler
    cfg = GriffinConfig.from_preset(Preset.RECURRENT_GEMMA_2B_V1)
    model = Griffin(cfg, device="cuda", dtype=torch.bfloat16,
                    vision=VisionConfig(image_size=224))

All arithmetic runs in the hand-written gfx950 kernels of
libcadence_hip.so (C ABI: include/cadence_kernels.h), bound as
torch.ops.cadence.*; there is no CPU fallback.
"""

from . import common
from . import layers
from . import modules
from . import griffin
from . import sampler
from . import vision
from . import checkpoint

ScanType = common.ScanType
TemporalBlockType = common.TemporalBlockType
Preset = common.Preset
GriffinConfig = common.GriffinConfig
VisionConfig = common.VisionConfig
ViTConfig = common.ViTConfig
rnn_scan = layers.rnn_scan
BlockDiagonalLinear = layers.BlockDiagonalLinear
RGLRU = layers.RGLRU
Conv1D = layers.Conv1D
RMSNorm = layers.RMSNorm
Einsum = layers.Einsum
RecurrentBlockCache = modules.RecurrentBlockCache
RecurrentBlock = modules.RecurrentBlock
AttentionBlockCache = modules.AttentionBlockCache
LocalAttentionBlock = modules.LocalAttentionBlock
ResidualBlockCache = modules.ResidualBlockCache
ResidualBlock = modules.ResidualBlock
MLPBlock = modules.MLPBlock
Embedder = modules.Embedder
Griffin = griffin.Griffin
Sampler = sampler.Sampler
SamplerOutput = sampler.SamplerOutput
VisionEncoder = vision.VisionEncoder
MLPProjector = vision.MLPProjector
load_params = checkpoint.load_params
load_griffin = checkpoint.load_griffin

__all__ = (
    "ScanType",
    "TemporalBlockType",
    "rnn_scan",
    "BlockDiagonalLinear",
    "RGLRU",
    "Conv1D",
    "RecurrentBlockCache",
    "RecurrentBlock",
    "AttentionBlockCache",
    "LocalAttentionBlock",
    "ResidualBlockCache",
    "ResidualBlock",
    "Preset",
    "GriffinConfig",
    "Griffin",
    "Sampler",
    "VisionEncoder",
    "MLPProjector",
    "VisionConfig",
)
