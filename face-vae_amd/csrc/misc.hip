// HBM-streaming kernels around the convs: layout changes, upsample backward, latent
// reparameterisation, KL / MSE / L1 reductions, spectral norm and multi-tensor Adam.
//
//   reparam : flatten_vae_nl convention (models.py:559-561), eps supplied by the caller
//   KL      : KLDivergenceLoss (losses.py:392)
//   MSE     : ReconLoss = nn.MSELoss (losses.py:396-403)
//   L1      : PerceptualLoss pixel term (losses.py:128,135)
//   SN      : torch/nn/utils/spectral_norm.py:62-113 (one power iteration per training fwd)
//   Adam    : torch.optim.Adam (logger.py:60)
#include <math.h>

#include <algorithm>

#include "common.h"

namespace {

constexpr int NTH = 256;
constexpr int RED_BLOCKS = 1024;   // first-stage blocks of the scalar loss reductions

int grid_for(long work, int cap = 8192) {
  long g = (work + NTH - 1) / NTH;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

template <typename T>
__device__ __forceinline__ float ldf(const T* p, long i) { return Elt<T>::to_f(p[i]); }

// -------------------------------------------------------------------------- layout
template <typename T>
__global__ void nchw_to_nhwc_kernel(const float* __restrict__ x, int N, int C, int HW, int ldc, T* out) {
  const int cg_n = (ldc + 7) / 8;
  const long total = (long)N * cg_n * HW;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int hw = (int)(e % HW);
    const long r = e / HW;
    const int cg = (int)(r % cg_n), n = (int)(r / cg_n);
    float f[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cg * 8 + j;
      f[j] = c < C ? x[((long)n * C + c) * HW + hw] : 0.f;
    }
    T* o = out + ((long)n * HW + hw) * ldc + cg * 8;
    if (cg * 8 + 8 <= ldc) {
      Chunk8<T> ch;
      ch.set8(f);
      ch.store(o);
    } else {
      for (int j = 0; j < 8 && cg * 8 + j < ldc; ++j) o[j] = Elt<T>::from_f(f[j]);
    }
  }
}

template <typename T>
__global__ void nhwc_to_nchw_kernel(const T* __restrict__ x, int N, int C, int HW, int ldc, float* out) {
  const int cg_n = (C + 7) / 8;
  const long total = (long)N * cg_n * HW;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int hw = (int)(e % HW);
    const long r = e / HW;
    const int cg = (int)(r % cg_n), n = (int)(r / cg_n);
    const T* ip = x + ((long)n * HW + hw) * ldc + cg * 8;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int c = cg * 8 + j;
      if (c < C) out[((long)n * C + c) * HW + hw] = Elt<T>::to_f(ip[j]);
    }
  }
}

template <typename TI, typename TO>
__global__ void cast_kernel(const TI* __restrict__ x, TO* y, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x)
    y[i] = Elt<TO>::from_f(Elt<TI>::to_f(x[i]));
}

// grid.y = source row (n*h + i), grid.x = (column j, 8-channel chunk) of that row
template <typename T>
__global__ void upsample_bwd_kernel(const T* __restrict__ g, int w, int C, int lgcpc, T* __restrict__ out) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= (w << lgcpc)) return;
  const int row = blockIdx.y;
  const int j = e >> lgcpc, c = (e & ((1 << lgcpc) - 1)) * 8;
  float acc[8] = {0, 0, 0, 0, 0, 0, 0, 0};
#pragma unroll
  for (int a = 0; a < 2; ++a)
#pragma unroll
    for (int b = 0; b < 2; ++b) {
      Chunk8<T> v;
      v.load(g + ((size_t)(2 * row + a) * (2 * w) + 2 * j + b) * C + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) acc[k] += v.get(k);
    }
  Chunk8<T> o;
  o.set8(acc);
  o.store(out + ((size_t)row * w + j) * C + c);
}

template <typename T>
__global__ void sigmoid_bwd_kernel(const float* __restrict__ dy, const float* __restrict__ y, int N, int C,
                                   int HW, int ldc, T* dpre) {
  const long total = (long)N * HW;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int n = (int)(e / HW), hw = (int)(e - (long)n * HW);
    T* o = dpre + e * ldc;
    for (int c = 0; c < ldc; ++c) {
      float v = 0.f;
      if (c < C) {
        const long i = ((long)n * C + c) * HW + hw;
        const float yy = y[i];
        v = dy[i] * yy * (1.f - yy);
      }
      o[c] = Elt<T>::from_f(v);
    }
  }
}

// ----------------------------------------------------------------- latent / losses
// grid.y = (n, 8-channel group), grid.x = hw (fastest: eps NCHW reads coalesce)
template <typename T>
__global__ void reparam_fwd_kernel(const T* __restrict__ h, const float* __restrict__ eps, int L, int HW,
                                   int cpc, T* __restrict__ mu, T* __restrict__ ls, T* __restrict__ z) {
  const int hw = blockIdx.x * blockDim.x + threadIdx.x;
  if (hw >= HW) return;
  const int n = blockIdx.y / cpc, cg = blockIdx.y - (blockIdx.y / cpc) * cpc;
  const size_t p = (size_t)n * HW + hw;
  Chunk8<T> m, s;
  m.load(h + p * 2 * L + cg * 8);
  s.load(h + p * 2 * L + L + cg * 8);
  const float* ep = eps + ((size_t)n * L + cg * 8) * HW + hw;
  float fz[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) fz[j] = m.get(j) + expf(s.get(j)) * ep[(size_t)j * HW];
  if (mu) {
    m.store(mu + p * L + cg * 8);
    s.store(ls + p * L + cg * 8);
  }
  Chunk8<T> o;
  o.set8(fz);
  o.store(z + p * L + cg * 8);
}

template <typename T>
__global__ void reparam_bwd_kernel(const T* __restrict__ h, const float* __restrict__ eps, int L, int HW, int cpc,
                                   const T* dz, const T* dmu, const T* dls, const float* klg, float kln,
                                   T* __restrict__ dh) {
  const int hw = blockIdx.x * blockDim.x + threadIdx.x;
  if (hw >= HW) return;
  const int n = blockIdx.y / cpc, cg = blockIdx.y - (blockIdx.y / cpc) * cpc;
  const size_t p = (size_t)n * HW + hw;
  const float kg = klg ? klg[0] * kln : 0.f;
  Chunk8<T> m, s, gz, gm, gs;
  if (klg) m.load(h + p * 2 * L + cg * 8); else m.zero();
  s.load(h + p * 2 * L + L + cg * 8);
  if (dz) gz.load(dz + p * L + cg * 8); else gz.zero();
  if (dmu) gm.load(dmu + p * L + cg * 8); else gm.zero();
  if (dls) gs.load(dls + p * L + cg * 8); else gs.zero();
  const float* ep = eps + ((size_t)n * L + cg * 8) * HW + hw;
  float om[8], os[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    const float ex = expf(s.get(j));
    om[j] = gz.get(j) + gm.get(j) + kg * m.get(j);
    os[j] = gz.get(j) * ex * ep[(size_t)j * HW] + gs.get(j) + kg * (ex * ex - 1.f);
  }
  Chunk8<T> a, b;
  a.set8(om);
  b.set8(os);
  a.store(dh + p * 2 * L + cg * 8);
  b.store(dh + p * 2 * L + L + cg * 8);
}

// Tiled forms (hw % 32 == 0): a block owns 32 pixels of one image x all L channels.  The
// eps tile [L][32] (NCHW fp32) is read coalesced into LDS and read back transposed, so the
// NHWC h / mu / logstd / z rows are touched as whole contiguous pixel rows.  The forward also
// writes the block's KL partial sum (losses.py:392, the sum before the mean) in fp64.
constexpr int RP_PX = 32;
template <typename T>
__global__ void __launch_bounds__(NTH) reparam_fwd_tiled(const T* __restrict__ h, const float* __restrict__ eps,
                                                          int L, int HW, T* __restrict__ mu, T* __restrict__ ls,
                                                          T* __restrict__ z, double* __restrict__ klpart) {
  extern __shared__ float es[];          // [L][RP_PX + 1]
  const int tpb = HW / RP_PX;
  const int n = blockIdx.x / tpb, hw0 = (blockIdx.x - n * tpb) * RP_PX;
  const int tid = threadIdx.x;
  const float* eb = eps + (size_t)n * L * HW + hw0;
  for (int f = tid; f < L * (RP_PX / 4); f += NTH) {
    const int c = f / (RP_PX / 4), px = (f - c * (RP_PX / 4)) * 4;
    const float4 v = *reinterpret_cast<const float4*>(eb + (size_t)c * HW + px);
    float* d = es + c * (RP_PX + 1) + px;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  const int G = L / 8;
  float kl = 0.f;
  for (int it = tid; it < RP_PX * G; it += NTH) {
    const int px = it / G, g = it - px * G;
    const size_t p = (size_t)n * HW + hw0 + px;
    Chunk8<T> m, s;
    m.load(h + p * 2 * L + g * 8);
    s.load(h + p * 2 * L + L + g * 8);
    float fz[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float mv = m.get(j), sv = s.get(j);
      const float ex = expf(sv);
      fz[j] = mv + ex * es[(g * 8 + j) * (RP_PX + 1) + px];
      kl += -0.5f - sv + 0.5f * mv * mv + 0.5f * ex * ex;
    }
    if (mu) {
      m.store(mu + p * L + g * 8);
      s.store(ls + p * L + g * 8);
    }
    Chunk8<T> o;
    o.set8(fz);
    o.store(z + p * L + g * 8);
  }
  if (klpart) {
    double acc = wave_sum_d((double)kl);
    __shared__ double sh[NTH / 64];
    if ((tid & 63) == 0) sh[tid >> 6] = acc;
    __syncthreads();
    if (tid == 0) {
      double t = 0;
      for (int i = 0; i < NTH / 64; ++i) t += sh[i];
      klpart[blockIdx.x] = t;
    }
  }
}

template <typename T>
__global__ void __launch_bounds__(NTH) reparam_bwd_tiled(const T* __restrict__ h, const float* __restrict__ eps,
                                                          int L, int HW, const T* dz, const T* dmu, const T* dls,
                                                          const float* klg, float kln, T* __restrict__ dh) {
  extern __shared__ float es[];
  const int tpb = HW / RP_PX;
  const int n = blockIdx.x / tpb, hw0 = (blockIdx.x - n * tpb) * RP_PX;
  const int tid = threadIdx.x;
  const float* eb = eps + (size_t)n * L * HW + hw0;
  for (int f = tid; f < L * (RP_PX / 4); f += NTH) {
    const int c = f / (RP_PX / 4), px = (f - c * (RP_PX / 4)) * 4;
    const float4 v = *reinterpret_cast<const float4*>(eb + (size_t)c * HW + px);
    float* d = es + c * (RP_PX + 1) + px;
    d[0] = v.x; d[1] = v.y; d[2] = v.z; d[3] = v.w;
  }
  __syncthreads();
  const int G = L / 8;
  const float kg = klg ? klg[0] * kln : 0.f;
  for (int it = tid; it < RP_PX * G; it += NTH) {
    const int px = it / G, g = it - px * G;
    const size_t p = (size_t)n * HW + hw0 + px;
    Chunk8<T> m, s, gz, gm, gs;
    if (klg) m.load(h + p * 2 * L + g * 8); else m.zero();
    s.load(h + p * 2 * L + L + g * 8);
    if (dz) gz.load(dz + p * L + g * 8); else gz.zero();
    if (dmu) gm.load(dmu + p * L + g * 8); else gm.zero();
    if (dls) gs.load(dls + p * L + g * 8); else gs.zero();
    float om[8], os[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const float ex = expf(s.get(j));
      om[j] = gz.get(j) + gm.get(j) + kg * m.get(j);
      os[j] = gz.get(j) * ex * es[(g * 8 + j) * (RP_PX + 1) + px] + gs.get(j) + kg * (ex * ex - 1.f);
    }
    Chunk8<T> a, b;
    a.set8(om);
    b.set8(os);
    a.store(dh + p * 2 * L + g * 8);
    b.store(dh + p * 2 * L + L + g * 8);
  }
}

// KL backward, 8 elements per thread: dmu = g mu / n, dlogstd = g (exp(2 logstd) - 1) / n
template <typename T>
__global__ void kl_bwd_vec_kernel(const T* __restrict__ mu, const T* __restrict__ ls, long n, const float* gout,
                                  T* dmu, T* dls) {
  const float g = gout[0] / (float)n;
  const long n8 = n / 8;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n8; i += (long)gridDim.x * blockDim.x) {
    Chunk8<T> m, s;
    m.load(mu + i * 8);
    s.load(ls + i * 8);
    float a[8], b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      a[j] = g * m.get(j);
      b[j] = g * (expf(2.f * s.get(j)) - 1.f);
    }
    if (dmu) { Chunk8<T> o; o.set8(a); o.store(dmu + i * 8); }
    if (dls) { Chunk8<T> o; o.set8(b); o.store(dls + i * 8); }
  }
}

// generic two-stage scalar mean: kind 0 = KL(mu, logstd), 1 = (a-b)^2, 2 = |a-b|
template <int KIND, typename T>
__global__ void loss_partial_kernel(const T* __restrict__ a, const T* __restrict__ b, long n, double* part) {
  double acc = 0;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float x = ldf(a, i), y = ldf(b, i);
    float v;
    if constexpr (KIND == 0) v = -0.5f - y + 0.5f * x * x + 0.5f * expf(2.f * y);
    else if constexpr (KIND == 1) v = (x - y) * (x - y);
    else v = fabsf(x - y);
    acc += v;
  }
  acc = wave_sum_d(acc);
  __shared__ double sh[NTH / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < NTH / 64; ++i) t += sh[i];
    part[blockIdx.x] = t;
  }
}

__global__ void loss_final_kernel(const double* part, int nparts, double count, float* out) {
  double acc = 0;
  for (int i = threadIdx.x; i < nparts; i += blockDim.x) acc += part[i];
  acc = wave_sum_d(acc);
  __shared__ double sh[NTH / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    double t = 0;
    for (int i = 0; i < NTH / 64; ++i) t += sh[i];
    out[0] = (float)(t / count);
  }
}

template <typename T>
__global__ void kl_bwd_kernel(const T* __restrict__ mu, const T* __restrict__ ls, long n, const float* gout,
                              T* dmu, T* dls) {
  const float g = gout[0] / (float)n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float m = ldf(mu, i), s = ldf(ls, i);
    if (dmu) dmu[i] = Elt<T>::from_f(g * m);
    if (dls) dls[i] = Elt<T>::from_f(g * (expf(2.f * s) - 1.f));
  }
}

template <int KIND>
__global__ void pair_bwd_kernel(const float* __restrict__ a, const float* __restrict__ b, long n,
                                const float* gout, float* da, float* db) {
  const float g = gout[0] / (float)n;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) {
    const float d = a[i] - b[i];
    float v;
    if constexpr (KIND == 1) v = 2.f * g * d;
    else v = d > 0.f ? g : (d < 0.f ? -g : 0.f);
    if (da) da[i] = v;
    if (db) db[i] = -v;
  }
}

// --------------------------------------------------------------------- spectral norm
// t = W^T u (cols): block = 64 columns x 4 row groups; per-block partial of |t|^2
__global__ void sn_wtu_kernel(const float* __restrict__ w, int rows, int cols, const float* __restrict__ u,
                              float* t, float* part) {
  const int j = blockIdx.x * 64 + (threadIdx.x & 63);
  const int rg = threadIdx.x >> 6;
  float acc = 0.f;
  if (j < cols)
    for (int i = rg; i < rows; i += 4) acc += w[(long)i * cols + j] * u[i];
  __shared__ float sh[4][64];
  sh[rg][threadIdx.x & 63] = acc;
  __syncthreads();
  float sq = 0.f;
  if (rg == 0) {
    const float v = sh[0][threadIdx.x] + sh[1][threadIdx.x] + sh[2][threadIdx.x] + sh[3][threadIdx.x];
    if (j < cols) t[j] = v;
    sq = j < cols ? v * v : 0.f;
    sq = wave_sum(sq);
    if (threadIdx.x == 0) part[blockIdx.x] = sq;
  }
}

// s = W v  (one wave per row), v = t / max(|t|, eps) when normalize (written out too)
__global__ void sn_wv_kernel(const float* __restrict__ w, int rows, int cols, const float* t,
                             const float* part, int nparts, int normalize, float* v, float* s) {
  float inv = 1.f;
  if (normalize) {
    float n2 = 0.f;
    for (int i = 0; i < nparts; ++i) n2 += part[i];
    inv = 1.f / fmaxf(sqrtf(n2), 1e-12f);
    for (int j = blockIdx.x * NTH + threadIdx.x; j < cols; j += gridDim.x * NTH) v[j] = t[j] * inv;
  }
  const float* vv = normalize ? t : v;
  const int lane = threadIdx.x & 63;
  const int row = blockIdx.x * (NTH / 64) + (threadIdx.x >> 6);
  if (row >= rows) return;
  float acc = 0.f;
  for (int j = lane; j < cols; j += 64) acc += w[(long)row * cols + j] * vv[j];
  acc = wave_sum(acc) * inv;
  if (lane == 0) s[row] = acc;
}

// u = s / max(|s|, eps) (power iteration) ; sigma = u . s
__global__ void sn_fin_kernel(const float* s, int rows, int update_u, float* u, float* sigma) {
  __shared__ float sh[NTH / 64];
  __shared__ float bc;
  float n2 = 0.f;
  for (int i = threadIdx.x; i < rows; i += NTH) n2 += s[i] * s[i];
  n2 = wave_sum(n2);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = n2;
  __syncthreads();
  if (threadIdx.x == 0) bc = 1.f / fmaxf(sqrtf(sh[0] + sh[1] + sh[2] + sh[3]), 1e-12f);
  __syncthreads();
  const float inv = bc;
  float d = 0.f;
  for (int i = threadIdx.x; i < rows; i += NTH) {
    float uu;
    if (update_u) {
      uu = s[i] * inv;
      u[i] = uu;
    } else {
      uu = u[i];
    }
    d += uu * s[i];
  }
  __syncthreads();
  d = wave_sum(d);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) sigma[0] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ void dot_partial_kernel(const float* __restrict__ a, const float* __restrict__ b, long n, float* part) {
  float acc = 0.f;
  for (long i = blockIdx.x * (long)NTH + threadIdx.x; i < n; i += (long)gridDim.x * NTH) acc += a[i] * b[i];
  acc = wave_sum(acc);
  __shared__ float sh[NTH / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ void sn_bwd_apply_kernel(const float* __restrict__ g, int rows, int cols, const float* u,
                                    const float* v, const float* sigma, const float* part, int nparts,
                                    float* out) {
  // <g, w> from the dot partials: every thread takes some, then a block reduction (a serial
  // loop in one thread was a chain of nparts dependent L2 round trips per block)
  __shared__ float red[NTH / 64];
  __shared__ float dot_s;
  float d = 0.f;
  for (int i = threadIdx.x; i < nparts; i += NTH) d += part[i];
  d = wave_sum(d);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < NTH / 64; ++i) t += red[i];
    dot_s = t;
  }
  __syncthreads();
  const float sg = sigma[0];
  const float c1 = 1.f / sg, c2 = dot_s / (sg * sg);
  const long n = (long)rows * cols;
  for (long e = blockIdx.x * (long)NTH + threadIdx.x; e < n; e += (long)gridDim.x * NTH) {
    const int i = (int)(e / cols), j = (int)(e - (long)i * cols);
    out[e] = g[e] * c1 - c2 * u[i] * v[j];
  }
}

// batched spectral-norm backward: grid (256, layers) partial dots, then grid (blocks, layers)
// apply; per layer the same partial count and order as fv_spectral_norm_bwd (bit-identical)
struct SnBwdMulti {
  int n;
  fv_sn_bwd_layer l[FV_SNB_MAX];
};
__global__ void sn_dot_multi_kernel(SnBwdMulti m, float* part) {
  const fv_sn_bwd_layer& L = m.l[blockIdx.y];
  const long n = (long)L.rows * L.cols;
  const int nb = (int)min((n + NTH - 1) / NTH, 256L);
  if ((int)blockIdx.x >= nb) return;
  float acc = 0.f;
  for (long i = blockIdx.x * (long)NTH + threadIdx.x; i < n; i += (long)nb * NTH) acc += L.g[i] * L.w[i];
  acc = wave_sum(acc);
  __shared__ float sh[NTH / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.y * 256 + blockIdx.x] = sh[0] + sh[1] + sh[2] + sh[3];
}

__global__ void sn_bwd_apply_multi_kernel(SnBwdMulti m, const float* part) {
  const fv_sn_bwd_layer& L = m.l[blockIdx.y];
  const long n = (long)L.rows * L.cols;
  const int nparts = (int)min((n + NTH - 1) / NTH, 256L);
  const float* pp = part + blockIdx.y * 256;
  __shared__ float red[NTH / 64];
  __shared__ float dot_s;
  float d = 0.f;
  for (int i = threadIdx.x; i < nparts; i += NTH) d += pp[i];
  d = wave_sum(d);
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = d;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int i = 0; i < NTH / 64; ++i) t += red[i];
    dot_s = t;
  }
  __syncthreads();
  const float sg = L.sigma[0];
  const float c1 = 1.f / sg, c2 = dot_s / (sg * sg);
  for (long e = blockIdx.x * (long)NTH + threadIdx.x; e < n; e += (long)gridDim.x * NTH) {
    const int i = (int)(e / L.cols), j = (int)(e - (long)i * L.cols);
    L.g[e] = L.g[e] * c1 - c2 * L.u[i] * L.v[j];
  }
}

// ---------------------------------------------------- batched spectral norm (all layers)
// One power iteration + sigma for every spectral-normed conv of the model in 4 launches
// (torch/nn/utils/spectral_norm.py:62-113 per layer): K1 partial W^T u over 64-row slices,
// K2 column sums -> t and |t|^2 partials, K3 s = W (t/|t|) one wave per row, K4 u = s/|s|,
// sigma = u.s (+ snapshots of u, v for the backward).  Layer descriptors live in a DEVICE
// table built once by the caller; blocks map to (layer, tile) through per-layer offsets.
struct SnDev {
  const float* w;
  float* u;
  float* v;
  float* sigma;
  float* usnap;
  float* vsnap;
  float* tp;      // [rs][cols] partials of W^T u
  float* t;       // [cols]
  float* part;    // [cdiv(cols, 256)] partial |t|^2
  float* s;       // [rows]
  int rows, cols;
  int b1, b2, b3; // first block of this layer in K1, K2, K3
};

__device__ __forceinline__ int sn_layer_of(const SnDev* L, int nl, int b, int which) {
  int l = 0;
  for (int i = 1; i < nl; ++i) {
    const int bi = which == 1 ? L[i].b1 : which == 2 ? L[i].b2 : L[i].b3;
    if (b >= bi) l = i;
  }
  return l;
}

__global__ void snb_wtu_kernel(const SnDev* __restrict__ L, int nl) {
  const int l = sn_layer_of(L, nl, blockIdx.x, 1);
  const SnDev d = L[l];
  const int ncb = (d.cols + 63) / 64;
  const int b = blockIdx.x - d.b1;
  const int rs = b / ncb, cb = b - rs * ncb;
  const int j = cb * 64 + (threadIdx.x & 63), rg = threadIdx.x >> 6;
  float acc = 0.f;
  if (j < d.cols) {
    const int r0 = rs * 64 + rg * 16;
#pragma unroll 4
    for (int i = r0; i < min(d.rows, r0 + 16); ++i) acc += d.w[(long)i * d.cols + j] * d.u[i];
  }
  __shared__ float sh[4][64];
  sh[rg][threadIdx.x & 63] = acc;
  __syncthreads();
  if (rg == 0 && j < d.cols)
    d.tp[(long)rs * d.cols + j] = (sh[0][threadIdx.x] + sh[1][threadIdx.x]) + (sh[2][threadIdx.x] + sh[3][threadIdx.x]);
}

__global__ void snb_colsum_kernel(const SnDev* __restrict__ L, int nl) {
  const int l = sn_layer_of(L, nl, blockIdx.x, 2);
  const SnDev d = L[l];
  const int b = blockIdx.x - d.b2;
  const int j = b * NTH + threadIdx.x;
  const int nrs = (d.rows + 63) / 64;
  float t = 0.f;
  if (j < d.cols) {
    for (int rs = 0; rs < nrs; ++rs) t += d.tp[(long)rs * d.cols + j];
    d.t[j] = t;
  }
  float sq = wave_sum(t * t);
  __shared__ float sh[NTH / 64];
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = sq;
  __syncthreads();
  if (threadIdx.x == 0) d.part[b] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

__global__ void snb_wv_kernel(const SnDev* __restrict__ L, int nl, int power_iter) {
  const int l = sn_layer_of(L, nl, blockIdx.x, 3);
  const SnDev d = L[l];
  const int b = blockIdx.x - d.b3;
  float inv = 1.f;
  const float* vv = d.v;
  if (power_iter) {
    float n2 = 0.f;
    for (int i = 0; i < (d.cols + NTH - 1) / NTH; ++i) n2 += d.part[i];
    inv = 1.f / fmaxf(sqrtf(n2), 1e-12f);
    vv = d.t;
    if (b == 0)
      for (int j = threadIdx.x; j < d.cols; j += NTH) {
        const float vj = d.t[j] * inv;
        d.v[j] = vj;
        d.vsnap[j] = vj;
      }
  } else if (b == 0) {
    for (int j = threadIdx.x; j < d.cols; j += NTH) d.vsnap[j] = d.v[j];
  }
  const int lane = threadIdx.x & 63;
  const int row = b * (NTH / 64) + (threadIdx.x >> 6);
  if (row >= d.rows) return;
  float acc = 0.f;
  for (int j = lane; j < d.cols; j += 64) acc += d.w[(long)row * d.cols + j] * vv[j];
  acc = wave_sum(acc) * inv;
  if (lane == 0) d.s[row] = acc;
}

__global__ void snb_fin_kernel(const SnDev* __restrict__ L, int power_iter) {
  const SnDev d = L[blockIdx.x];
  __shared__ float sh[NTH / 64];
  __shared__ float bc;
  float n2 = 0.f;
  for (int i = threadIdx.x; i < d.rows; i += NTH) n2 += d.s[i] * d.s[i];
  n2 = wave_sum(n2);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = n2;
  __syncthreads();
  if (threadIdx.x == 0) bc = 1.f / fmaxf(sqrtf((sh[0] + sh[1]) + (sh[2] + sh[3])), 1e-12f);
  __syncthreads();
  const float inv = bc;
  float dd = 0.f;
  for (int i = threadIdx.x; i < d.rows; i += NTH) {
    const float uu = power_iter ? d.s[i] * inv : d.u[i];
    if (power_iter) d.u[i] = uu;
    d.usnap[i] = uu;
    dd += uu * d.s[i];
  }
  __syncthreads();
  dd = wave_sum(dd);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = dd;
  __syncthreads();
  if (threadIdx.x == 0) d.sigma[0] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// ------------------------------------------------------------------------------ Adam
__global__ void adam_kernel(const fv_adam_tensor* __restrict__ ts, const int* __restrict__ blocks, float omb1,
                            float b2, float omb2, float eps, float step_size, float bc2_sqrt) {
  const int t = blocks[2 * blockIdx.x], ch = blocks[2 * blockIdx.x + 1];
  const fv_adam_tensor d = ts[t];
  const long base = (long)ch * FV_ADAM_CHUNK;
  const long end = min(d.numel, base + FV_ADAM_CHUNK);
  for (long i = base + threadIdx.x; i < end; i += NTH) {
    const float g = d.grad[i];
    float m = d.exp_avg[i], v = d.exp_avg_sq[i];
    m = m + omb1 * (g - m);                 // exp_avg.lerp_(grad, 1 - beta1)
    v = v * b2 + omb2 * g * g;              // exp_avg_sq.mul_(beta2).addcmul_(g, g, 1 - beta2)
    d.exp_avg[i] = m;
    d.exp_avg_sq[i] = v;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    d.param[i] = d.param[i] - step_size * (m / denom);
  }
}

// device-step variant: one lane advances the step and writes the coefficients (fp64 math,
// as fv_adam_step computes them on the host), then adam_dev_kernel reads them
__global__ void adam_coef_kernel(double* step, float* coef, double lr, double beta1, double beta2) {
  if (threadIdx.x != 0) return;
  const double t = step[0] + 1.0;
  step[0] = t;
  const double bc1 = 1.0 - pow(beta1, t);
  const double bc2 = 1.0 - pow(beta2, t);
  coef[0] = (float)(lr / bc1);
  coef[1] = (float)sqrt(bc2);
}

__global__ void adam_dev_kernel(const fv_adam_tensor* __restrict__ ts, const int* __restrict__ blocks, float omb1,
                                float b2, float omb2, float eps, const float* __restrict__ coef) {
  const float step_size = coef[0], bc2_sqrt = coef[1];
  const int t = blocks[2 * blockIdx.x], ch = blocks[2 * blockIdx.x + 1];
  const fv_adam_tensor d = ts[t];
  const long base = (long)ch * FV_ADAM_CHUNK;
  const long end = min(d.numel, base + FV_ADAM_CHUNK);
  for (long i = base + threadIdx.x; i < end; i += NTH) {
    const float g = d.grad[i];
    float m = d.exp_avg[i], v = d.exp_avg_sq[i];
    m = m + omb1 * (g - m);
    v = v * b2 + omb2 * g * g;
    d.exp_avg[i] = m;
    d.exp_avg_sq[i] = v;
    const float denom = sqrtf(v) / bc2_sqrt + eps;
    d.param[i] = d.param[i] - step_size * (m / denom);
  }
}

}  // namespace

extern "C" {

int fv_nchw_to_nhwc(int dtype_out, const float* x, int n, int c, int hw, int ldc, void* out, void* stream) {
  FV_REQUIRE(x && out && ldc >= c, "bad args");
  const long work = (long)n * ((ldc + 7) / 8) * hw;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_out == FV_BF16)
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<bf16>, dim3(grid_for(work)), dim3(NTH), 0, s, x, n, c, hw, ldc, (bf16*)out);
  else
    hipLaunchKernelGGL(nchw_to_nhwc_kernel<float>, dim3(grid_for(work)), dim3(NTH), 0, s, x, n, c, hw, ldc, (float*)out);
  return fv_check_launch("nchw_to_nhwc");
}

int fv_nhwc_to_nchw(int dtype_in, const void* x, int n, int c, int hw, int ldc, float* out, void* stream) {
  FV_REQUIRE(x && out && ldc >= c, "bad args");
  const long work = (long)n * ((c + 7) / 8) * hw;
  hipStream_t s = (hipStream_t)stream;
  if (dtype_in == FV_BF16)
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<bf16>, dim3(grid_for(work)), dim3(NTH), 0, s, (const bf16*)x, n, c, hw, ldc, out);
  else
    hipLaunchKernelGGL(nhwc_to_nchw_kernel<float>, dim3(grid_for(work)), dim3(NTH), 0, s, (const float*)x, n, c, hw, ldc, out);
  return fv_check_launch("nhwc_to_nchw");
}

int fv_cast(int dtype_in, const void* x, int dtype_out, void* y, long count, void* stream) {
  FV_REQUIRE(x && y, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int g = grid_for(count);
  if (dtype_in == FV_F32 && dtype_out == FV_BF16)
    hipLaunchKernelGGL((cast_kernel<float, bf16>), dim3(g), dim3(NTH), 0, s, (const float*)x, (bf16*)y, count);
  else if (dtype_in == FV_BF16 && dtype_out == FV_F32)
    hipLaunchKernelGGL((cast_kernel<bf16, float>), dim3(g), dim3(NTH), 0, s, (const bf16*)x, (float*)y, count);
  else if (dtype_in == FV_F32 && dtype_out == FV_F32)
    hipLaunchKernelGGL((cast_kernel<float, float>), dim3(g), dim3(NTH), 0, s, (const float*)x, (float*)y, count);
  else
    hipLaunchKernelGGL((cast_kernel<bf16, bf16>), dim3(g), dim3(NTH), 0, s, (const bf16*)x, (bf16*)y, count);
  return fv_check_launch("cast");
}

int fv_upsample2x_bwd(int dtype, const void* g, int n, int h_src, int w_src, int c, void* out, void* stream) {
  FV_REQUIRE(g && out && c % 8 == 0 && fv_ilog2(c / 8) >= 0, "upsample bwd: channels must be 8 * a power of two");
  FV_REQUIRE(n * h_src <= 65535 && (long)n * h_src * w_src * 4 * c < (1L << 31), "upsample bwd: too large");
  const int lgcpc = fv_ilog2(c / 8);
  const dim3 grid(fv_cdiv((long)w_src << lgcpc, NTH), n * h_src);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(upsample_bwd_kernel<bf16>, grid, dim3(NTH), 0, s, (const bf16*)g, w_src, c, lgcpc, (bf16*)out);
  else
    hipLaunchKernelGGL(upsample_bwd_kernel<float>, grid, dim3(NTH), 0, s, (const float*)g, w_src, c, lgcpc,
                       (float*)out);
  return fv_check_launch("upsample2x_bwd");
}

int fv_sigmoid_bwd_to_nhwc(int dtype_out, const float* dy, const float* y, int n, int c, int hw, int ldc,
                           void* dpre, void* stream) {
  FV_REQUIRE(dy && y && dpre && ldc >= c, "bad args");
  hipStream_t s = (hipStream_t)stream;
  const long work = (long)n * hw;
  if (dtype_out == FV_BF16)
    hipLaunchKernelGGL(sigmoid_bwd_kernel<bf16>, dim3(grid_for(work)), dim3(NTH), 0, s, dy, y, n, c, hw, ldc,
                       (bf16*)dpre);
  else
    hipLaunchKernelGGL(sigmoid_bwd_kernel<float>, dim3(grid_for(work)), dim3(NTH), 0, s, dy, y, n, c, hw, ldc,
                       (float*)dpre);
  return fv_check_launch("sigmoid_bwd");
}

size_t fv_loss_ws_bytes(void) { return RED_BLOCKS * sizeof(double); }

size_t fv_reparam_ws_bytes(int n, int L, int hw) {
  (void)L;
  return (size_t)(hw % RP_PX == 0 ? (long)n * (hw / RP_PX) : 1) * sizeof(double);
}

static size_t reparam_lds(int L) { return (size_t)L * (RP_PX + 1) * sizeof(float); }

int fv_reparam_tiled(int L, int hw) { return hw % RP_PX == 0 && reparam_lds(L) <= 64 * 1024; }

int fv_reparam_kl_fwd(int dtype, const void* h, const float* eps, int n, int L, int hw, void* mu, void* logstd,
                      void* z, float* kl, void* ws, void* stream) {
  FV_REQUIRE(h && eps && z && L % 8 == 0 && !mu == !logstd, "reparam: bad args (L %% 8 == 0)");
  hipStream_t s = (hipStream_t)stream;
  if (fv_reparam_tiled(L, hw)) {
    FV_REQUIRE(!kl || ws, "reparam: KL output needs the workspace");
    const int nb = n * (hw / RP_PX);
    double* part = kl ? (double*)ws : nullptr;
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(reparam_fwd_tiled<bf16>, dim3(nb), dim3(NTH), reparam_lds(L), s, (const bf16*)h, eps, L, hw,
                         (bf16*)mu, (bf16*)logstd, (bf16*)z, part);
    else
      hipLaunchKernelGGL(reparam_fwd_tiled<float>, dim3(nb), dim3(NTH), reparam_lds(L), s, (const float*)h, eps, L,
                         hw, (float*)mu, (float*)logstd, (float*)z, part);
    int st = fv_check_launch("reparam_fwd_tiled");
    if (st || !kl) return st;
    hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(NTH), 0, s, part, nb, (double)n * L * hw, kl);
    return fv_check_launch("reparam_kl_final");
  }
  FV_REQUIRE(n * (L / 8) <= 65535, "reparam: too many (image, channel-group) rows");
  const dim3 grid(fv_cdiv(hw, NTH), n * (L / 8));
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(reparam_fwd_kernel<bf16>, grid, dim3(NTH), 0, s, (const bf16*)h, eps, L, hw, L / 8,
                       (bf16*)mu, (bf16*)logstd, (bf16*)z);
  else
    hipLaunchKernelGGL(reparam_fwd_kernel<float>, grid, dim3(NTH), 0, s, (const float*)h, eps, L, hw, L / 8,
                       (float*)mu, (float*)logstd, (float*)z);
  int st = fv_check_launch("reparam_fwd");
  if (st || !kl) return st;
  FV_REQUIRE(ws && mu, "reparam: the KL of an untiled shape needs the workspace and the mu/logstd outputs");
  return fv_kl_fwd(dtype, mu, logstd, (long)n * L * hw, kl, ws, stream);
}

int fv_reparam_fwd(int dtype, const void* h, const float* eps, int n, int L, int hw, void* mu, void* logstd,
                   void* z, void* stream) {
  return fv_reparam_kl_fwd(dtype, h, eps, n, L, hw, mu, logstd, z, nullptr, nullptr, stream);
}

int fv_reparam_kl_bwd(int dtype, const void* h, const float* eps, int n, int L, int hw, const void* dz,
                      const void* dmu, const void* dlogstd, const float* kl_grad, void* dh, void* stream) {
  FV_REQUIRE(h && eps && dh && L % 8 == 0, "reparam bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  const float kln = (float)(1.0 / ((double)n * L * hw));
  if (fv_reparam_tiled(L, hw)) {
    const int nb = n * (hw / RP_PX);
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(reparam_bwd_tiled<bf16>, dim3(nb), dim3(NTH), reparam_lds(L), s, (const bf16*)h, eps, L, hw,
                         (const bf16*)dz, (const bf16*)dmu, (const bf16*)dlogstd, kl_grad, kln, (bf16*)dh);
    else
      hipLaunchKernelGGL(reparam_bwd_tiled<float>, dim3(nb), dim3(NTH), reparam_lds(L), s, (const float*)h, eps, L,
                         hw, (const float*)dz, (const float*)dmu, (const float*)dlogstd, kl_grad, kln, (float*)dh);
    return fv_check_launch("reparam_bwd_tiled");
  }
  FV_REQUIRE(n * (L / 8) <= 65535, "reparam: too many (image, channel-group) rows");
  const dim3 grid(fv_cdiv(hw, NTH), n * (L / 8));
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(reparam_bwd_kernel<bf16>, grid, dim3(NTH), 0, s, (const bf16*)h, eps, L, hw, L / 8,
                       (const bf16*)dz, (const bf16*)dmu, (const bf16*)dlogstd, kl_grad, kln, (bf16*)dh);
  else
    hipLaunchKernelGGL(reparam_bwd_kernel<float>, grid, dim3(NTH), 0, s, (const float*)h, eps, L, hw, L / 8,
                       (const float*)dz, (const float*)dmu, (const float*)dlogstd, kl_grad, kln, (float*)dh);
  return fv_check_launch("reparam_bwd");
}

int fv_reparam_bwd(int dtype, const void* h, const float* eps, int n, int L, int hw, const void* dz,
                   const void* dmu, const void* dlogstd, void* dh, void* stream) {
  return fv_reparam_kl_bwd(dtype, h, eps, n, L, hw, dz, dmu, dlogstd, nullptr, dh, stream);
}

static int reduce_scalar(int kind, int dtype, const void* a, const void* b, long count, float* loss, void* ws,
                         hipStream_t s) {
  FV_REQUIRE(a && b && loss && ws && count > 0, "loss: bad args");
  const int g = grid_for(count, RED_BLOCKS);
  double* part = (double*)ws;
  if (kind == 0) {
    if (dtype == FV_BF16)
      hipLaunchKernelGGL((loss_partial_kernel<0, bf16>), dim3(g), dim3(NTH), 0, s, (const bf16*)a, (const bf16*)b, count, part);
    else
      hipLaunchKernelGGL((loss_partial_kernel<0, float>), dim3(g), dim3(NTH), 0, s, (const float*)a, (const float*)b, count, part);
  } else if (kind == 1) {
    hipLaunchKernelGGL((loss_partial_kernel<1, float>), dim3(g), dim3(NTH), 0, s, (const float*)a, (const float*)b, count, part);
  } else {
    hipLaunchKernelGGL((loss_partial_kernel<2, float>), dim3(g), dim3(NTH), 0, s, (const float*)a, (const float*)b, count, part);
  }
  int st = fv_check_launch("loss_partial");
  if (st) return st;
  hipLaunchKernelGGL(loss_final_kernel, dim3(1), dim3(NTH), 0, s, part, g, (double)count, loss);
  return fv_check_launch("loss_final");
}

int fv_kl_fwd(int dtype, const void* mu, const void* logstd, long count, float* loss, void* ws, void* stream) {
  return reduce_scalar(0, dtype, mu, logstd, count, loss, ws, (hipStream_t)stream);
}

int fv_kl_bwd(int dtype, const void* mu, const void* logstd, long count, const float* gout, void* dmu,
              void* dlogstd, void* stream) {
  FV_REQUIRE(mu && logstd && gout, "kl bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  if (count % 8 == 0) {
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(kl_bwd_vec_kernel<bf16>, dim3(grid_for(count / 8)), dim3(NTH), 0, s, (const bf16*)mu,
                         (const bf16*)logstd, count, gout, (bf16*)dmu, (bf16*)dlogstd);
    else
      hipLaunchKernelGGL(kl_bwd_vec_kernel<float>, dim3(grid_for(count / 8)), dim3(NTH), 0, s, (const float*)mu,
                         (const float*)logstd, count, gout, (float*)dmu, (float*)dlogstd);
    return fv_check_launch("kl_bwd");
  }
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(kl_bwd_kernel<bf16>, dim3(grid_for(count)), dim3(NTH), 0, s, (const bf16*)mu, (const bf16*)logstd,
                       count, gout, (bf16*)dmu, (bf16*)dlogstd);
  else
    hipLaunchKernelGGL(kl_bwd_kernel<float>, dim3(grid_for(count)), dim3(NTH), 0, s, (const float*)mu,
                       (const float*)logstd, count, gout, (float*)dmu, (float*)dlogstd);
  return fv_check_launch("kl_bwd");
}

int fv_mse_fwd(const float* a, const float* b, long count, float* loss, void* ws, void* stream) {
  return reduce_scalar(1, FV_F32, a, b, count, loss, ws, (hipStream_t)stream);
}
int fv_l1_fwd(const float* a, const float* b, long count, float* loss, void* ws, void* stream) {
  return reduce_scalar(2, FV_F32, a, b, count, loss, ws, (hipStream_t)stream);
}
int fv_mse_bwd(const float* a, const float* b, long count, const float* gout, float* da, float* db, void* stream) {
  FV_REQUIRE(a && b && gout, "mse bwd: bad args");
  hipLaunchKernelGGL(pair_bwd_kernel<1>, dim3(grid_for(count)), dim3(NTH), 0, (hipStream_t)stream, a, b, count, gout,
                     da, db);
  return fv_check_launch("mse_bwd");
}
int fv_l1_bwd(const float* a, const float* b, long count, const float* gout, float* da, float* db, void* stream) {
  FV_REQUIRE(a && b && gout, "l1 bwd: bad args");
  hipLaunchKernelGGL(pair_bwd_kernel<2>, dim3(grid_for(count)), dim3(NTH), 0, (hipStream_t)stream, a, b, count, gout,
                     da, db);
  return fv_check_launch("l1_bwd");
}

size_t fv_spectral_norm_ws_bytes(int rows, int cols) {
  return ((size_t)cols + rows + 2 * NTH + 64) * sizeof(float);
}

int fv_spectral_norm_fwd(const float* w, int rows, int cols, float* u, float* v, float* sigma, int power_iter,
                         void* ws, void* stream) {
  FV_REQUIRE(w && u && v && sigma && ws && rows > 0 && cols > 0, "spectral norm: bad args");
  hipStream_t s = (hipStream_t)stream;
  float* t = (float*)ws;
  float* sv = t + cols;
  float* part = sv + rows;
  const int nparts = fv_cdiv(cols, 64);
  FV_REQUIRE(nparts <= 2 * NTH, "spectral norm: too many columns");
  if (power_iter) {
    hipLaunchKernelGGL(sn_wtu_kernel, dim3(nparts), dim3(NTH), 0, s, w, rows, cols, u, t, part);
    int st = fv_check_launch("sn_wtu");
    if (st) return st;
  }
  hipLaunchKernelGGL(sn_wv_kernel, dim3(fv_cdiv(rows, NTH / 64)), dim3(NTH), 0, s, w, rows, cols, t, part, nparts,
                     power_iter, v, sv);
  int st = fv_check_launch("sn_wv");
  if (st) return st;
  hipLaunchKernelGGL(sn_fin_kernel, dim3(1), dim3(NTH), 0, s, sv, rows, power_iter, u, sigma);
  return fv_check_launch("sn_fin");
}

int fv_spectral_norm_bwd(const float* w, const float* g_sn, int rows, int cols, const float* u, const float* v,
                         const float* sigma, float* g_orig, void* ws, void* stream) {
  FV_REQUIRE(w && g_sn && u && v && sigma && g_orig && ws, "spectral norm bwd: bad args");
  hipStream_t s = (hipStream_t)stream;
  float* part = (float*)ws;
  const long n = (long)rows * cols;
  const int nb = (int)std::min<long>(fv_cdiv(n, NTH), 256);
  hipLaunchKernelGGL(dot_partial_kernel, dim3(nb), dim3(NTH), 0, s, g_sn, w, n, part);
  int st = fv_check_launch("sn_dot");
  if (st) return st;
  hipLaunchKernelGGL(sn_bwd_apply_kernel, dim3(grid_for(n, 2048)), dim3(NTH), 0, s, g_sn, rows, cols, u, v, sigma,
                     part, nb, g_orig);
  return fv_check_launch("sn_bwd");
}

int fv_spectral_norm_bwd_multi(int n, const fv_sn_bwd_layer* layers, float* ws, void* stream) {
  FV_REQUIRE(n >= 1 && n <= FV_SNB_MAX && layers && ws, "spectral norm bwd multi: bad args");
  SnBwdMulti m{};
  m.n = n;
  long maxn = 0;
  for (int i = 0; i < n; ++i) {
    const fv_sn_bwd_layer& L = layers[i];
    FV_REQUIRE(L.w && L.g && L.u && L.v && L.sigma && L.rows > 0 && L.cols > 0, "spectral norm bwd multi: layer %d", i);
    m.l[i] = L;
    maxn = std::max(maxn, (long)L.rows * L.cols);
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(sn_dot_multi_kernel, dim3(256, n), dim3(NTH), 0, s, m, ws);
  int st = fv_check_launch("sn_dot_multi");
  if (st) return st;
  hipLaunchKernelGGL(sn_bwd_apply_multi_kernel, dim3(grid_for(maxn, 2048), n), dim3(NTH), 0, s, m, (const float*)ws);
  return fv_check_launch("sn_bwd_multi");
}

size_t fv_spectral_norm_batch_ws_floats(const fv_sn_layer* layers, int nlayers) {
  size_t n = 0;
  for (int i = 0; i < nlayers; ++i) {
    const int r = layers[i].rows, c = layers[i].cols;
    n += (size_t)((r + 63) / 64) * c + c + (c + NTH - 1) / NTH + r;
  }
  return n;
}

size_t fv_spectral_norm_batch_table_bytes(int nlayers) { return (size_t)nlayers * sizeof(SnDev); }

int fv_spectral_norm_batch_build(const fv_sn_layer* layers, int nlayers, float* ws, void* table_host,
                                 int* nblocks3) {
  FV_REQUIRE(layers && nlayers > 0 && ws && table_host && nblocks3, "sn batch build: bad args");
  SnDev* T = (SnDev*)table_host;
  int b1 = 0, b2 = 0, b3 = 0;
  float* p = ws;
  for (int i = 0; i < nlayers; ++i) {
    const fv_sn_layer& s = layers[i];
    FV_REQUIRE(s.w && s.u && s.v && s.sigma && s.usnap && s.vsnap && s.rows > 0 && s.cols > 0, "sn layer %d", i);
    SnDev d{};
    d.w = s.w; d.u = s.u; d.v = s.v; d.sigma = s.sigma; d.usnap = s.usnap; d.vsnap = s.vsnap;
    d.rows = s.rows; d.cols = s.cols;
    const int nrs = (s.rows + 63) / 64;
    d.tp = p; p += (size_t)nrs * s.cols;
    d.t = p; p += s.cols;
    d.part = p; p += (s.cols + NTH - 1) / NTH;
    d.s = p; p += s.rows;
    d.b1 = b1; b1 += nrs * ((s.cols + 63) / 64);
    d.b2 = b2; b2 += (s.cols + NTH - 1) / NTH;
    d.b3 = b3; b3 += (s.rows + NTH / 64 - 1) / (NTH / 64);
    T[i] = d;
  }
  nblocks3[0] = b1;
  nblocks3[1] = b2;
  nblocks3[2] = b3;
  return FV_OK;
}

int fv_spectral_norm_fwd_batch(const void* table_dev, int nlayers, const int* nblocks3, int power_iter,
                               void* stream) {
  FV_REQUIRE(table_dev && nlayers > 0 && nblocks3, "sn batch: bad args");
  hipStream_t s = (hipStream_t)stream;
  const SnDev* L = (const SnDev*)table_dev;
  int st;
  if (power_iter) {
    hipLaunchKernelGGL(snb_wtu_kernel, dim3(nblocks3[0]), dim3(NTH), 0, s, L, nlayers);
    if ((st = fv_check_launch("snb_wtu"))) return st;
    hipLaunchKernelGGL(snb_colsum_kernel, dim3(nblocks3[1]), dim3(NTH), 0, s, L, nlayers);
    if ((st = fv_check_launch("snb_colsum"))) return st;
  }
  hipLaunchKernelGGL(snb_wv_kernel, dim3(nblocks3[2]), dim3(NTH), 0, s, L, nlayers, power_iter);
  if ((st = fv_check_launch("snb_wv"))) return st;
  hipLaunchKernelGGL(snb_fin_kernel, dim3(nlayers), dim3(NTH), 0, s, L, power_iter);
  return fv_check_launch("snb_fin");
}

int fv_adam_step(const fv_adam_tensor* tensors, const int* blocks, int nblocks, double lr, double beta1,
                 double beta2, double eps, long step, void* stream) {
  FV_REQUIRE(tensors && blocks && nblocks > 0 && step > 0, "adam: bad args");
  // scalar coefficients in double on the host, as torch.optim.Adam computes them in Python
  const double bc1 = 1.0 - pow(beta1, (double)step);
  const double bc2 = 1.0 - pow(beta2, (double)step);
  hipLaunchKernelGGL(adam_kernel, dim3(nblocks), dim3(NTH), 0, (hipStream_t)stream, tensors, blocks,
                     (float)(1.0 - beta1), (float)beta2, (float)(1.0 - beta2), (float)eps, (float)(lr / bc1),
                     (float)sqrt(bc2));
  return fv_check_launch("adam");
}

int fv_adam_step_dev(const fv_adam_tensor* tensors, const int* blocks, int nblocks, double lr, double beta1,
                     double beta2, double eps, double* step_dev, float* coef_ws, void* stream) {
  FV_REQUIRE(tensors && blocks && nblocks > 0 && step_dev && coef_ws, "adam_dev: bad args");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(adam_coef_kernel, dim3(1), dim3(64), 0, s, step_dev, coef_ws, lr, beta1, beta2);
  int st = fv_check_launch("adam_coef");
  if (st) return st;
  hipLaunchKernelGGL(adam_dev_kernel, dim3(nblocks), dim3(NTH), 0, s, tensors, blocks, (float)(1.0 - beta1),
                     (float)beta2, (float)(1.0 - beta2), (float)eps, coef_ws);
  return fv_check_launch("adam_dev");
}

int fv_copy_h2d_async(void* dst, const void* src_pinned, size_t bytes, void* stream) {
  FV_REQUIRE(dst && src_pinned, "copy_h2d: bad args");
  hipError_t e = hipMemcpyAsync(dst, src_pinned, bytes, hipMemcpyHostToDevice, (hipStream_t)stream);
  if (e != hipSuccess) {
    fv_set_error("copy_h2d: %s", hipGetErrorString(e));
    return (int)e;
  }
  return FV_OK;
}

}  // extern "C"
