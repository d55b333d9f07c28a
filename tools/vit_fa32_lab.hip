// Lab build of the 32x32x16 ViT attention kernel (csrc/vit_fa32.hip) with
// its measurement variants (the LAB bits) and ring depths, for
// tools/vit_fa32_lab.py.  Not part of the product library.
#include "vit_fa32_kernel.hip"

template <int HD, int NB, int LAB>
static void fa32_lab_launch(const void* qkv, void* out, int64_t B, int64_t N, int64_t H,
                            hipStream_t st) {
  const int64_t ntq = (N + 31) / 32, nqb = (ntq + 3) / 4;
  const int64_t units = B * H * nqb;
  const unsigned g = (unsigned)std::min<int64_t>((units + 7) / 8 * 8, (LAB & 64) ? 768 : 512);
  hipLaunchKernelGGL((vit_fa32_kernel<HD, NB, true, LAB>), dim3(g),
                     dim3(256), 0, st, static_cast<const u16*>(qkv), static_cast<u16*>(out),
                     (int)B, (int)N, (int)H, (int)nqb, 1.0f);
}

#define LAB_CASES(HD_, NB_)                                              \
  switch (lab) {                                                         \
    case 1: fa32_lab_launch<HD_, NB_, 1>(qkv, out, B, N, H, st); break;   \
    case 2: fa32_lab_launch<HD_, NB_, 2>(qkv, out, B, N, H, st); break;   \
    case 4: fa32_lab_launch<HD_, NB_, 4>(qkv, out, B, N, H, st); break;   \
    case 6: fa32_lab_launch<HD_, NB_, 6>(qkv, out, B, N, H, st); break;   \
    case 8: fa32_lab_launch<HD_, NB_, 8>(qkv, out, B, N, H, st); break;   \
    case 16: fa32_lab_launch<HD_, NB_, 16>(qkv, out, B, N, H, st); break; \
    case 7: fa32_lab_launch<HD_, NB_, 7>(qkv, out, B, N, H, st); break;   \
    case 24: fa32_lab_launch<HD_, NB_, 24>(qkv, out, B, N, H, st); break; \
    case 30: fa32_lab_launch<HD_, NB_, 30>(qkv, out, B, N, H, st); break; \
    case 31: fa32_lab_launch<HD_, NB_, 31>(qkv, out, B, N, H, st); break; \
    case 32: fa32_lab_launch<HD_, NB_, 32>(qkv, out, B, N, H, st); break; \
    case 64: fa32_lab_launch<HD_, NB_, 64>(qkv, out, B, N, H, st); break; \
    case 96: fa32_lab_launch<HD_, NB_, 96>(qkv, out, B, N, H, st); break; \
    default: return -1;                                                  \
  }

extern "C" int fa32_lab(const void* qkv, void* out, int64_t B, int64_t N, int64_t H,
                        int64_t hd, int lab, int nb, void* stream) {
  hipStream_t st = static_cast<hipStream_t>(stream);
  // lab 0: the product launch (q already scaled), whatever nb says
  if (lab == 0) return vit_fa32_attention_launch(qkv, out, B, N, H, hd, 1, stream);
  if (hd == 64 && nb == 3) { LAB_CASES(64, 3) }
  else if (hd == 64 && nb == 4) { LAB_CASES(64, 4) }
  else if (hd == 72 && nb == 3) { LAB_CASES(72, 3) }
  else if (hd == 72 && nb == 4) { LAB_CASES(72, 4) }
  else return -1;
  return (int)hipGetLastError();
}
