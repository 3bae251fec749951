// Shared device/host helpers for libfacevae (gfx950 / CDNA4 only).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/facevae.h"

typedef __bf16 bf16;
typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define FV_LDS __attribute__((address_space(3)))

// ------------------------------------------------------------------------------------
// host-side error plumbing (thread-local message, never abort)
// ------------------------------------------------------------------------------------
void fv_set_error(const char* fmt, ...);
int fv_check_launch(const char* what);

#define FV_REQUIRE(cond, ...)                  \
  do {                                         \
    if (!(cond)) {                             \
      fv_set_error(__VA_ARGS__);               \
      return FV_E_BADARG;                      \
    }                                          \
  } while (0)

static inline int fv_ilog2(int v) {
  int l = 0;
  while ((1 << l) < v) ++l;
  return ((1 << l) == v) ? l : -1;
}
static inline int fv_cdiv(long a, long b) { return (int)((a + b - 1) / b); }

// ------------------------------------------------------------------------------------
// element helpers: T is float (fp32 parity mode) or bf16 (fast mode)
// ------------------------------------------------------------------------------------
template <typename T> struct Elt;
template <> struct Elt<float> {
  static __device__ __forceinline__ float to_f(float v) { return v; }
  static __device__ __forceinline__ float from_f(float v) { return v; }
};
template <> struct Elt<bf16> {
  static __device__ __forceinline__ float to_f(bf16 v) { return (float)v; }
  static __device__ __forceinline__ bf16 from_f(float v) { return (bf16)v; }
};

// 8 consecutive elements moved as raw bits (16 B for bf16, 32 B for f32)
template <typename T> struct Chunk8;
template <> struct Chunk8<bf16> {
  uint4 raw;
  __device__ __forceinline__ void load(const bf16* p) { raw = *reinterpret_cast<const uint4*>(p); }
  __device__ __forceinline__ void store(bf16* p) const { *reinterpret_cast<uint4*>(p) = raw; }
  __device__ __forceinline__ void zero() { raw = make_uint4(0, 0, 0, 0); }
  __device__ __forceinline__ float get(int j) const {
    const uint32_t w = (&raw.x)[j >> 1];
    const uint32_t b = (j & 1) ? (w & 0xffff0000u) : (w << 16);
    return __uint_as_float(b);
  }
  __device__ __forceinline__ void set8(const float* f) {
    bf16 t[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) t[j] = (bf16)f[j];
    raw = *reinterpret_cast<const uint4*>(t);
  }
};
template <> struct Chunk8<float> {
  float4 a, b;
  __device__ __forceinline__ void load(const float* p) {
    a = reinterpret_cast<const float4*>(p)[0];
    b = reinterpret_cast<const float4*>(p)[1];
  }
  __device__ __forceinline__ void store(float* p) const {
    reinterpret_cast<float4*>(p)[0] = a;
    reinterpret_cast<float4*>(p)[1] = b;
  }
  __device__ __forceinline__ void zero() { a = b = make_float4(0.f, 0.f, 0.f, 0.f); }
  __device__ __forceinline__ float get(int j) const { return j < 4 ? (&a.x)[j] : (&b.x)[j - 4]; }
  __device__ __forceinline__ void set8(const float* f) {
    a = make_float4(f[0], f[1], f[2], f[3]);
    b = make_float4(f[4], f[5], f[6], f[7]);
  }
};

// ReLU / LeakyReLU, 0 <= slope <= 1 (ReLU 0, LeakyReLU 0.2: modules.py:41-47): max(v, v * slope)
// is v for v > 0 and v * slope otherwise, bit for bit (signed zeros and NaN included; only
// -inf at slope 0 differs: -inf, not NaN) -- one v_mul + one v_max instead of a compare-select.
// The entry points reject slopes outside [0, 1] (fv_slope_ok)
__device__ __forceinline__ float fv_act(float v, float slope) { return fmaxf(v, v * slope); }
static inline bool fv_slope_ok(float slope) { return slope >= 0.f && slope <= 1.f; }

// wave-level reductions (wave64)
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}
// sum over each row of 16 lanes, result in every lane of the row: 4 DPP adds (quad swaps,
// half-row and row mirrors) instead of 4 ds_bpermute round trips
template <int CTRL>
__device__ __forceinline__ float dpp_f(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_mov_dpp(__builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ float row16_sum(float v) {
  v += dpp_f<0xB1>(v);    // quad_perm [1,0,3,2]
  v += dpp_f<0x4E>(v);    // quad_perm [2,3,0,1]
  v += dpp_f<0x141>(v);   // row_half_mirror
  v += dpp_f<0x140>(v);   // row_mirror
  return v;
}
__device__ __forceinline__ float wave_max(float v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o, 64));
  return v;
}
__device__ __forceinline__ double wave_sum_d(double v) {
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o, 64);
  return v;
}

// ------------------------------------------------------------------------------------
// unsigned division by a run-time constant (host precomputes m, s); exact for n < 2^31
// ------------------------------------------------------------------------------------
struct FastDiv {
  uint32_t m, s;
};
static inline FastDiv make_fastdiv(uint32_t d) {
  uint32_t s = 0;
  while ((1u << s) < d) ++s;
  const uint64_t m = ((1ull << 32) * ((1ull << s) - d)) / d + 1;
  return {(uint32_t)m, s};
}
__device__ __forceinline__ uint32_t fdiv(uint32_t n, FastDiv f) { return (__umulhi(n, f.m) + n) >> f.s; }

// ------------------------------------------------------------------------------------
// fp8 (e4m3) delayed-scaling sites, shared by the quantize passes (conv.hip) and the BN passes
// that write an fp8 copy of their output (bn.hip).  site = uint32[FP8_SITE]: [0, 16) amax
// history (float bits), [16] amax of the call in flight (float bits, atomicMax: max is
// order-free, so deterministic), [17] history write index, [18] dq of the call in flight.
// ------------------------------------------------------------------------------------
constexpr int FP8_SITE = 32, FP8_HIST = 16;

// largest power of two s with amax * s <= 448
__device__ __forceinline__ float pow2_scale_of(float amax) {
  if (!(amax > 0.f) || !isfinite(amax)) return 1.f;
  return exp2f(floorf(log2f(448.f / amax)));
}
__device__ __forceinline__ uint32_t pack4_fp8(float a, float b, float c, float d) {
  int v = __builtin_amdgcn_cvt_pk_fp8_f32(a, b, 0, false);
  v = __builtin_amdgcn_cvt_pk_fp8_f32(c, d, v, true);
  return (uint32_t)v;
}
__device__ __forceinline__ float site_hist_max(const unsigned* st) {
  float m = 0.f;
#pragma unroll
  for (int i = 0; i < FP8_HIST; ++i) m = fmaxf(m, __uint_as_float(st[i]));
  return m;
}
// 8 values -> 8 e4m3 bytes with the call's scale s (saturating at +-448); m = running amax of
// the unscaled values
__device__ __forceinline__ uint2 q8_pack(const float* v, float s, float& m) {
  float q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    m = fmaxf(m, fabsf(v[j]));
    q[j] = fminf(fmaxf(v[j] * s, -448.f), 448.f);
  }
  uint2 o;
  o.x = pack4_fp8(q[0], q[1], q[2], q[3]);
  o.y = pack4_fp8(q[4], q[5], q[6], q[7]);
  return o;
}
// block (blockDim.x threads, a multiple of 64, no early exits) amax -> the site's in-flight slot
__device__ __forceinline__ void q8_block_amax(float m, unsigned* st) {
  m = wave_max(m);
  __shared__ float red[16];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) {
    float r = 0.f;
    for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = fmaxf(r, red[w]);
    atomicMax(st + 16, __float_as_uint(r));
  }
}
