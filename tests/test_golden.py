"""Golden fixtures (tests/golden/*.safetensors, made by tests/golden/make_golden.py).

CPU: the oracle still reproduces the committed vectors (elementwise ops
bit-exact; matmul-containing outputs to a tight tolerance, since CPU GEMM
blocking may differ between hosts).  GPU: the HIP path against the same
committed vectors, with the per-kernel bars of tests/test_kernels_gpu.py
(scan and conv bit-exact) and the end-to-end bars of SURVEY §8c (cosine
>= 0.999 on logits, first greedy token identical).
"""

import os

import pytest
import torch
from safetensors import safe_open
from safetensors.torch import load_file

from conftest import cosine, rel_l2
from oracle import griffin_ref as R

import cadence

GOLD = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")
BF = torch.bfloat16


def _load(name):
  path = os.path.join(GOLD, name)
  with safe_open(path, "pt") as f:
    meta = f.metadata() or {}
  return load_file(path), meta


@pytest.fixture(scope="module")
def kern():
  return _load("kernels.safetensors")[0]


def _mg():
  import importlib.util
  spec = importlib.util.spec_from_file_location(
      "make_golden", os.path.join(GOLD, "make_golden.py"))
  mod = importlib.util.module_from_spec(spec)
  spec.loader.exec_module(mod)
  return mod


def _params(fixture, meta, prefix, cfg, vision, seed):
  p = _mg().golden_params(cfg, vision=vision, seed=seed)
  keys = meta["param_keys"].split(",")
  assert sorted(p) == keys, "state-dict keys drifted from the fixture"
  sums = torch.tensor([p[k].double().sum().item() for k in keys],
                      dtype=torch.float64)
  torch.testing.assert_close(sums, fixture[f"{prefix}.param_sums"],
                             rtol=0, atol=0, msg="seeded weights drifted")
  return p


# ------------------------------------------------------------------ CPU

def test_golden_oracle_kernels(kern):
  k = kern
  reset = k["scan.reset"].bool()
  y, h = R.rnn_scan(k["scan.x"], k["scan.a"], reset, k["scan.h0"])
  assert torch.equal(y, k["scan.y"]) and torch.equal(h, k["scan.h_last"])
  y, h = R.rnn_scan(k["scan.x"], k["scan.a"], reset, None)
  assert torch.equal(y, k["scan.y_noh0"]) and torch.equal(h, k["scan.h_last_noh0"])
  y, h = R.rnn_scan(k["scan1.x"], k["scan1.a"],
                    torch.zeros(4, 1, dtype=torch.bool), k["scan1.h0"])
  assert torch.equal(y, k["scan1.y"]) and torch.equal(h, k["scan1.h_last"])
  for compat in (True, False):
    yc, cc = R.conv1d(k["conv.x"], k["conv.pos"], k["conv.w"], k["conv.b"],
                      None, compat=compat)
    assert torch.equal(yc, k[f"conv.y_compat{int(compat)}"])
    assert torch.equal(cc, k[f"conv.cache_compat{int(compat)}"])
  b = k["convd.x"].shape[0]
  yd, cd = R.conv1d(k["convd.x"], torch.full((b, 1), 9, dtype=torch.int32),
                    k["conv.w"], k["conv.b"], k["convd.cache"])
  assert torch.equal(yd, k["convd.y"]) and torch.equal(cd, k["convd.cache_out"])
  torch.testing.assert_close(R.rms_norm(k["rms.x"], k["rms.scale"]).float(),
                             k["rms.y"].float(), rtol=1e-2, atol=1e-2)


def test_golden_oracle_text_model():
  mg = _mg()
  f, meta = _load("text_model.safetensors")
  cfg = mg.text_config()
  p = _params(f, meta, "text", cfg, None, 31)
  logits, _ = R.griffin_forward(p, cfg, f["text.tokens"].long(), f["text.pos"])
  assert cosine(logits, f["text.logits"]) > 0.99999
  gtok, _ = R.greedy_sample(p, cfg, f["text.tokens"].long(),
                            f["text.greedy_tokens"].shape[1])
  assert torch.equal(gtok.to(torch.int32), f["text.greedy_tokens"])


def test_golden_oracle_multimodal():
  mg = _mg()
  f, meta = _load("mm_model.safetensors")
  cfg, vis = mg.text_config(), mg.tiny_vision()
  p = _params(f, meta, "mm", cfg, vis, 41)
  feats = R.vision_encoder(f["mm.pixels"], p, vis)
  assert rel_l2(feats, f["mm.features"]) < 1e-5
  img = R.projector(feats, p)
  logits, _ = R.griffin_forward(p, cfg, f["mm.tokens"].long(), f["mm.pos"],
                                image_tokens=img)
  assert cosine(logits, f["mm.logits"]) > 0.99999


# ------------------------------------------------------------------ GPU

@pytest.mark.gpu
def test_golden_hip_kernels(dev, kern):
  k = kern
  reset = k["scan.reset"].bool()
  y, h = cadence.rnn_scan(k["scan.x"].to(dev), k["scan.a"].to(dev),
                          reset.to(dev), k["scan.h0"].to(dev))
  assert torch.equal(y.cpu(), k["scan.y"]) and torch.equal(h.cpu(), k["scan.h_last"])
  y, h = cadence.rnn_scan(k["scan.x"].to(dev), k["scan.a"].to(dev),
                          reset.to(dev), None)
  assert torch.equal(y.cpu(), k["scan.y_noh0"])
  assert torch.equal(h.cpu(), k["scan.h_last_noh0"])
  y, h = cadence.rnn_scan(k["scan1.x"].to(dev), k["scan1.a"].to(dev),
                          torch.zeros(4, 1, dtype=torch.bool, device=dev),
                          k["scan1.h0"].to(dev))
  assert torch.equal(y.cpu(), k["scan1.y"]) and torch.equal(h.cpu(), k["scan1.h_last"])
  e = k["conv.x"].shape[-1]
  for compat in (True, False):
    conv = cadence.Conv1D(e, 4, device=dev, dtype=BF, compat=compat)
    with torch.no_grad():
      conv.w.copy_(k["conv.w"])
      conv.b.copy_(k["conv.b"])
    yc, cc = conv(k["conv.x"].to(dev), k["conv.pos"].to(dev))
    assert torch.equal(yc.cpu(), k[f"conv.y_compat{int(compat)}"])
    assert torch.equal(cc.cpu(), k[f"conv.cache_compat{int(compat)}"])
  b = k["convd.x"].shape[0]
  yd, cd = conv(k["convd.x"].to(dev),
                torch.full((b, 1), 9, dtype=torch.int32, device=dev),
                k["convd.cache"].to(dev))
  assert torch.equal(yd.cpu(), k["convd.y"]) and torch.equal(cd.cpu(), k["convd.cache_out"])
  norm = cadence.RMSNorm(k["rms.x"].shape[-1], device=dev, dtype=BF)
  with torch.no_grad():
    norm.scale.copy_(k["rms.scale"])
  torch.testing.assert_close(norm(k["rms.x"].to(dev)).float().cpu(),
                             k["rms.y"].float(), rtol=2e-2, atol=2e-2)


class _Vocab:
  def pad_id(self): return 0
  def bos_id(self): return 2
  def eos_id(self): return 1


def _gpu_model(dev, p, cfg, vision=None):
  m = cadence.Griffin(cfg, device=dev, dtype=BF, vision=vision)
  m.load_state_dict({k: v.to(dev) for k, v in p.items()})
  return m


@pytest.mark.gpu
def test_golden_hip_text_model(dev):
  mg = _mg()
  f, meta = _load("text_model.safetensors")
  cfg = mg.text_config()
  m = _gpu_model(dev, _params(f, meta, "text", cfg, None, 31), cfg)
  tok, pos = f["text.tokens"], f["text.pos"]
  with torch.no_grad():
    got, _ = m(tok.to(dev), pos.to(dev))
  assert cosine(got, f["text.logits"]) > 0.999
  assert rel_l2(got, f["text.logits"]) < 3e-2
  steps = f["text.greedy_tokens"].shape[1]
  s = cadence.Sampler(m, _Vocab())
  st = s.generate(tok, torch.full((tok.shape[0],), tok.shape[1],
                                  dtype=torch.int32), steps, return_logits=True)
  assert torch.equal(st.tokens_buffer[:, 0].cpu(), f["text.greedy_tokens"][:, 0])
  assert cosine(st.logits_buffer[:, 0].cpu(), f["text.greedy_logits"][:, 0]) > 0.999
  agree = (st.tokens_buffer.cpu() == f["text.greedy_tokens"]).float().mean().item()
  assert agree >= 0.75, agree


@pytest.mark.gpu
def test_golden_hip_multimodal(dev):
  mg = _mg()
  f, meta = _load("mm_model.safetensors")
  cfg, vis = mg.text_config(), mg.tiny_vision()
  m = _gpu_model(dev, _params(f, meta, "mm", cfg, vis, 41), cfg, vis)
  px = f["mm.pixels"].to(dev)
  with torch.no_grad():
    feats = m.vis_encoder.encode(px)
    assert rel_l2(feats, f["mm.features"]) < 1e-2
    assert rel_l2(m.projector(feats), f["mm.image_tokens"]) < 2e-2
    got, _ = m(f["mm.tokens"].to(dev), f["mm.pos"].to(dev), images=px)
  assert got.shape == f["mm.logits"].shape
  assert cosine(got, f["mm.logits"]) > 0.999


# ------------------------------------------------- image preprocessing

def _decode(name):
  from cadence import image_io
  return image_io.decode_rgb(os.path.join(GOLD, "images", name))


def test_golden_images_pillow_and_restatement():
  """The reference's own test JPEGs: Pillow's bicubic resize (the
  reference's transform) reproduces the fixture, and so does the oracle's
  restatement of its resampler that the HIP kernel follows."""
  f, _ = _load("images.safetensors")
  for name in ("car2.jpg", "german.jpg"):
    arr = _decode(name)
    assert int(arr.astype("int64").sum()) == int(f[f"{name}.decoded_sum"][0])
    for size in (224, 336):
      want = f[f"{name}.{size}"]
      got = R.pil_resize_to_tensor(arr, size)
      assert torch.equal(got, want.permute(2, 0, 1).float().div(255))
      if size == 224:
        assert torch.equal(torch.from_numpy(R.pil_resample_np(arr, size)), want)


@pytest.mark.gpu
def test_golden_images_hip_resize(dev):
  from cadence import image_io
  f, _ = _load("images.safetensors")
  names = ("car2.jpg", "german.jpg")
  for size in (224, 336):
    got = image_io.load_images([os.path.join(GOLD, "images", n) for n in names],
                               size, dev).cpu()
    assert got.shape == (2, 3, size, size)
    for i, n in enumerate(names):
      want = f[f"{n}.{size}"].permute(2, 0, 1).float().div(255)
      assert torch.equal(got[i], want), (n, size)
