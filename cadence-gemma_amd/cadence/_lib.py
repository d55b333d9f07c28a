"""Loader for libcadence_hip.so, the C ABI of include/cadence_kernels.h.

The library is built in-tree (`make -C cadence-gemma_amd`) and loaded with
ctypes after torch, so it binds to the HIP runtime torch already mapped (one
runtime per process; verified by `hip_runtimes_loaded`).  There is no CPU
fallback: if the library is missing, every op raises.
"""

from __future__ import annotations

import ctypes
import os
import threading

import torch  # noqa: F401  (load torch's HIP runtime first)

_HERE = os.path.dirname(os.path.abspath(__file__))
# CADENCE_LIB_PATH: the host-ASan build of the same C-ABI
# (tools/asan_host.sh, CPU-only contract tests); unset everywhere else
LIB_PATH = os.environ.get("CADENCE_LIB_PATH") or os.path.join(_HERE, "libcadence_hip.so")
ABI_VERSION = 18

_lock = threading.Lock()
_lib: ctypes.CDLL | None = None

P = ctypes.c_void_p
I64 = ctypes.c_int64
I32 = ctypes.c_int
F32 = ctypes.c_float

# name -> argtypes (restype int unless listed in _RESTYPE)
_SIGS: dict[str, list] = {
    "cadence_abi_version": [],
    "cadence_gemm_workspace_bytes": [I64, I64, I64, I64],
    "cadence_gemm_tile_rows": [I64, I64, I64, I64],
    "cadence_gemm_big_splits": [I64, I64, I64, I64],
    "cadence_gemm_set_engine": [I32],
    "cadence_gemm_engine": [I64, I64, I64, I64],
    "cadence_gemm_linear": [P, I64, P, I64, P, P, I64, P, I64, I64, I64, I64,
                            I32, I64, I64, I64, P, I64, P],
    "cadence_gemm_gated_gelu": [P, I64, P, I64, P, P, P, I64, I64, I64, I64, P,
                                I64, I32, F32, P],
    "cadence_rglru_gates": [P, I64, P, I64, P, P, P, P, P, P, I64, I64, I64, I64,
                            P, I64, P],
    "cadence_rglru_gates_stream_plan": [P, I64, P, I64, I64, I64, I64],
    "cadence_rglru_scan": [P, I64, P, P, P, P, P, P, P, I64, P, I64, P, I64, I64,
                           I64, I64, P],
    "cadence_rglru_scan_plan": [P, I64, P, I64, I64, I64, I64, I64, I64],
    "cadence_gemm_rmsnorm_workspace_bytes": [I64, I64, I64],
    "cadence_qkv_rope_decode": [P, I64, P, I64, P, P, P, P, I64, I64, I64, I64, P,
                                I64, I32, F32, P],
    "cadence_qkv_rope_prefill": [P, I64, P, I64, P, P, P, P, I64, I64, I64, I64, P,
                                 I64, P],
    "cadence_gemm_linear_conv1d": [P, I64, P, I64, P, P, I64, I64, I64, I64, I64,
                                   P, P, P, I64, I32, F32, P],
    "cadence_gemm_linear_residual_rows": [P, I64, P, I64, P, P, I64, P, I64, P,
                                          I64, I64, I64, P, I64, P, P],
    "cadence_gemm_linear_rmsnorm": [P, I64, P, I64, P, P, I64, P, I64, I64, I64,
                                    I64, P, F32, P, I64, P, I64, P],
    "cadence_recurrent_decode_front_plan": [I64, I64, I64, I64, I64],
    "cadence_recurrent_decode_front": [P, P, P, P, I64, I64, I64, P, P, P, I32, F32, P, P,
                                       P, P, P, P, P, I64, I64, P, P, P],
    "cadence_rglru_step": [P, I64, P, I64, P, P, P, P, P, P, I64, P, I64, I64,
                           I64, I64, P, I64, P],
    "cadence_gemm_vit_residual": [P, I64, P, I64, P, P, P, I64, I64, I64, I64,
                                  P, I64, P],
    "cadence_gemm_patch_embed": [P, I64, P, I64, P, P, P, I64, I64, I64, I64,
                                 I64, I64, P, I64, P],
    "cadence_logits_argmax": [P, I64, P, I64, I64, I64, I64, F32, P, P, P, I64, P],
    "cadence_logits_scratch_bytes": [I64, I64, I64],
    "cadence_gemm_logits": [P, I64, P, I64, I64, I64, I64, F32, P, I64, P, I64, P],
    "cadence_rmsnorm": [P, I64, P, P, I64, I64, I64, F32, P],
    "cadence_layernorm": [P, I64, P, P, P, I64, I64, I64, F32, P],
    "cadence_embed": [P, P, P, I64, I64, I64, I64, F32, I64, I64, I64, P],
    "cadence_embed_packed": [P, P, P, I64, P, I64, I64, I64, F32, P],
    "cadence_logits_argmax_tail": [P, I64, P, I64, I64, I64, I64, F32, P, P, I64, P, P],
    "cadence_conv1d": [P, I64, P, P, P, P, P, I64, P, I64, I64, I64, I64, I32,
                       P],
    "cadence_rnn_scan": [P, I64, P, I64, P, P, P, I64, P, I64, P, I64, I64, I64,
                         P, I64, P],
    "cadence_rnn_scan_workspace_bytes": [I64, I64, I64],
    "cadence_segment_info": [P, P, P, I64, I64, P],
    "cadence_rope_qkv": [P, I64, P, P, P, P, I64, I64, I64, P, I64, P],
    "cadence_rope_table": [P, I64, I64, P],
    "cadence_local_attention": [P, P, P, P, P, P, I64, I64, I64, I64, I64, P],
    "cadence_kv_cache_fill": [P, P, P, P, P, P, I64, I64, I64, I64, P],
    "cadence_local_attention_decode": [P, P, P, P, P, P, P, I64, I64, I64, I64,
                                       I64, P, I64, P, P],
    "cadence_local_attention_decode_workspace_bytes": [I64, I64],
    "cadence_im2col_normalize": [P, P, I64, I64, I64, I64, P, P, P],
    "cadence_vit_prefix": [P, P, I64, I64, I64, I64, P],
    "cadence_vit_attention": [P, P, I64, I64, I64, I64, P],
    "cadence_vit_attention_kernel": [I64, I64],
    "cadence_vit_features": [P, P, I64, I64, I64, I64, I64, I64, P],
    "cadence_resize_bicubic": [P, I64, P, I64, I64, I64, I64, I64, P, P, I64, P,
                               P],
    "cadence_splice_positions": [P, P, I64, I64, I64, P],
    "cadence_local_attention_cached": [P, P, P, P, P, P, P, I64, I64, I64, I64,
                                       I64, P],
    "cadence_kv_ring_update": [P, P, P, P, P, I64, I64, I64, P],
    "cadence_copy_batched": [P, I64, P],
    "cadence_decode_advance": [P, P, I64, P, P, P, P, I32, I32, I32, I64, P],
}
_RESTYPE = {
    "cadence_gemm_workspace_bytes": I64,
    "cadence_local_attention_decode_workspace_bytes": I64,
    "cadence_gemm_rmsnorm_workspace_bytes": I64,
    "cadence_logits_scratch_bytes": I64,
    "cadence_rnn_scan_workspace_bytes": I64,
}


class CopyDesc(ctypes.Structure):
  """CadenceCopyDesc (cadence_kernels.h): one row-strided copy region."""
  _fields_ = [("src", P), ("dst", P), ("rows", I64), ("row_bytes", I64),
              ("src_stride", I64), ("dst_stride", I64)]


class DecodeTail(ctypes.Structure):
  """CadenceDecodeTail (cadence_kernels.h): the decode step's bookkeeping and
  next-input rows for cadence_logits_argmax_tail."""
  _fields_ = [("tokens_out", P), ("ld_out", I64), ("step", P), ("positions", P),
              ("cur_out", P), ("done", P), ("eos_id", I32), ("pad_id", I32),
              ("eos_from", I32), ("counter", P), ("embed", P), ("vocab", I64),
              ("scale", F32), ("x_out", P), ("ldx_out", I64), ("packed_out", P)]


class KernelLibraryMissing(RuntimeError):
  pass


def _declare(lib: ctypes.CDLL) -> None:
  for name, args in _SIGS.items():
    fn = getattr(lib, name)
    fn.argtypes = args
    fn.restype = _RESTYPE.get(name, I32)


def load() -> ctypes.CDLL:
  """Returns the loaded kernel library; raises if it is not built."""
  global _lib
  if _lib is not None:
    return _lib
  with _lock:
    if _lib is None:
      if not os.path.exists(LIB_PATH):
        raise KernelLibraryMissing(
            f"{LIB_PATH} is missing: build it with `make -C "
            f"{os.path.dirname(_HERE)}` (hipcc --offload-arch=gfx950). The "
            "MI355X path has no CPU fallback.")
      lib = ctypes.CDLL(LIB_PATH, mode=ctypes.RTLD_GLOBAL)
      _declare(lib)
      v = lib.cadence_abi_version()
      if v != ABI_VERSION:
        raise KernelLibraryMissing(f"ABI mismatch: library {v}, host {ABI_VERSION}")
      _lib = lib
  return _lib


def exported_symbols() -> list[str]:
  return sorted(_SIGS)


def hip_runtimes_loaded() -> list[str]:
  """Paths of every libamdhip64 mapped into this process."""
  found = set()
  with open("/proc/self/maps") as f:
    for line in f:
      if "libamdhip64" in line:
        found.add(line.split()[-1])
  return sorted(found)


def check(status: int, what: str) -> None:
  if status != 0:
    raise RuntimeError(f"{what} failed with hipError {status}")
