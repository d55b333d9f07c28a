"""roctx ranges around the hot path's phases (tracing row).

The reference has no tracing on its torch path (only unused `import time`
lines, recurrentgemma/torch/layers.py:29 and a timing note at :366).  Here
`torch.cuda.nvtx` (roctx on ROCm: torch's libroctx64) marks the vision
towers, the projector, each residual block by type, the RG-LRU scan and the
sampler's prefill / decode phases, so `rocprofv3 --marker-trace` (or
`--kernel-trace` + markers) attributes kernels to them.  Off by default (a
range costs host time per call); on with CADENCE_ROCTX=1 or `enable()`.
Ranges are host-side: none are pushed while a hipGraph is being captured.
"""

from __future__ import annotations

import contextlib
import os

import torch

_ON = os.environ.get("CADENCE_ROCTX", "0") == "1"


def enable(on: bool = True) -> None:
  global _ON
  _ON = bool(on)


def enabled() -> bool:
  return _ON


@contextlib.contextmanager
def trace(name: str):
  if not _ON or (torch.cuda.is_available() and
                 torch.cuda.is_current_stream_capturing()):
    yield
    return
  torch.cuda.nvtx.range_push(name)
  try:
    yield
  finally:
    torch.cuda.nvtx.range_pop()
