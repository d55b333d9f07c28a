"""Shared test setup.

`-m "not gpu"`: oracle KATs, config/API surface, C-ABI load + exports,
gloo multi-process data-parallel logic.  `-m gpu`: kernel and model parity
against the CPU oracle (oracle/), on an MI355X.
"""

import os
import sys

import pytest
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for p in (os.path.join(ROOT, "cadence-gemma_amd"), ROOT):
  if p not in sys.path:
    sys.path.insert(0, p)


def pytest_configure(config):
  config.addinivalue_line("markers", "gpu: needs an MI355X (HIP) device")


@pytest.fixture(scope="session")
def dev():
  if not torch.cuda.is_available():
    pytest.skip("no GPU")
  return torch.device("cuda", 0)


def assert_close_bf16(got, want, rtol=2e-2, atol=2e-2, min_equal=None, what=""):
  got = got.detach().float().cpu()
  want = want.detach().float().cpu()
  assert got.shape == want.shape, (what, got.shape, want.shape)
  torch.testing.assert_close(got, want, rtol=rtol, atol=atol, msg=what)
  if min_equal is not None:
    frac = (got == want).float().mean().item()
    assert frac >= min_equal, f"{what}: only {frac:.4f} bitwise equal"


def cosine(a, b):
  a = a.detach().float().cpu().flatten()
  b = b.detach().float().cpu().flatten()
  return float(torch.dot(a, b) / (a.norm() * b.norm() + 1e-30))


def rel_l2(a, b):
  a = a.detach().float().cpu()
  b = b.detach().float().cpu()
  return float((a - b).norm() / (b.norm() + 1e-30))
