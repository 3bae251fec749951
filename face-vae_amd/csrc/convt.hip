// Generic ConvTranspose2dELR (models_utils.py:404-516) for gfx950: any kernel size / stride /
// padding, fp32 (parity mode) or bf16 operands, NHWC activations.  Direct kernels (VALU, fp32
// accumulation): the FaceVAE-relevant geometry k4 s2 p1 at power-of-two sizes runs on the
// sub-pixel MFMA kernels of conv.hip instead (fv_convt_supported).
//   convt_eff_weight   W_eff = gain * [1 / max(||W[:, o]||, 1e-12)] * W   (F.normalize over dims
//                      [0, 2, 3] when demod, models_utils.py:461-470; gain 429-433)
//   convt_direct_fwd   out[n][oh][ow][o] = b + sum_{i, r, s} x[n][ih][iw][i] W_eff[i][o][r][s],
//                      oh = ih * S - P + r  (F.conv_transpose2d, models_utils.py:497-498)
//   convt_direct_dgrad dx[n][ih][iw][i] = sum_{o, r, s} dy[n][ih*S-P+r][iw*S-P+s][o] W_eff[i][o][r][s]
//   convt_direct_wgrad G[i][o][r][s] = sum x[n][ih][iw][i] dy[n][ih*S-P+r][iw*S-P+s][o]
//   convt_weight_grad  G -> dL/dW through the demodulation and gain
//   chan_scale         y[n][p][c] = x[n][p][c] * a[n][c] + b[n][c] and its backward (the
//                      per-sample modulation x * (affine(w) * 0.1 + 1) and demod factor,
//                      models_utils.py:486-495, applied to activations instead of weights)
#include "common.h"

namespace {

__device__ __forceinline__ float ldv(const float* p) { return *p; }
__device__ __forceinline__ float ldv(const bf16* p) { return (float)*p; }

__global__ void __launch_bounds__(64) convt_norm_any_kernel(const float* __restrict__ w, int cin, int cout, int kk,
                                                            float* inv) {
  const int co = blockIdx.x, l = threadIdx.x;
  float s = 0.f;
  for (int e = l; e < cin * kk; e += 64) {
    const float v = w[((long)(e / kk) * cout + co) * kk + (e % kk)];
    s += v * v;
  }
  s = wave_sum(s);
  if (l == 0) inv[co] = 1.f / fmaxf(sqrtf(s), 1e-12f);
}

__global__ void __launch_bounds__(256) convt_eff_weight_kernel(const float* __restrict__ w, const float* inv,
                                                               float gain, int cout, int kk, long n, float* we) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= n) return;
  const int co = (int)((e / kk) % cout);
  we[e] = w[e] * (inv ? gain * inv[co] : gain);
}

// in place, one wave per output channel: G = dL/dW_eff -> dL/dW (see conv.hip convt_weight_bwd)
__global__ void __launch_bounds__(64) convt_weight_grad_kernel(const float* __restrict__ w, const float* inv,
                                                               float gain, float* g, int cin, int cout, int kk) {
  const int co = blockIdx.x, l = threadIdx.x;
  const float iv = inv ? inv[co] : 1.f;
  float dot = 0.f;
  if (inv && iv < 1e12f) {
    for (int e = l; e < cin * kk; e += 64) {
      const long a = ((long)(e / kk) * cout + co) * kk + (e % kk);
      dot += w[a] * iv * g[a];
    }
    dot = wave_sum(dot);
  }
  for (int e = l; e < cin * kk; e += 64) {
    const long a = ((long)(e / kk) * cout + co) * kk + (e % kk);
    g[a] = gain * iv * (g[a] - (inv ? w[a] * iv * dot : 0.f));
  }
}

struct CtArgs {
  int N, Hi, Wi, Ho, Wo, Ci, Co, ldx, ldy, K, S, P;
};

// one output element per thread
template <typename T>
__global__ void __launch_bounds__(256) convt_direct_fwd(const T* __restrict__ x, const float* __restrict__ we,
                                                        const float* bias, T* __restrict__ y, CtArgs a) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long tot = (long)a.N * a.Ho * a.Wo * a.Co;
  if (e >= tot) return;
  const int o = (int)(e % a.Co);
  const long p = e / a.Co;
  const int ow = (int)(p % a.Wo), oh = (int)((p / a.Wo) % a.Ho);
  const long n = p / ((long)a.Wo * a.Ho);
  float acc = bias ? bias[o] : 0.f;
  for (int r = 0; r < a.K; ++r) {
    const int th = oh + a.P - r;
    if (th < 0 || th % a.S) continue;
    const int ih = th / a.S;
    if (ih >= a.Hi) continue;
    for (int s = 0; s < a.K; ++s) {
      const int tw = ow + a.P - s;
      if (tw < 0 || tw % a.S) continue;
      const int iw = tw / a.S;
      if (iw >= a.Wi) continue;
      const T* xp = x + ((n * a.Hi + ih) * a.Wi + iw) * a.ldx;
      const float* wp = we + (long)o * a.K * a.K + r * a.K + s;
      for (int i = 0; i < a.Ci; ++i) acc = fmaf(ldv(xp + i), wp[(long)i * a.Co * a.K * a.K], acc);
    }
  }
  y[p * a.ldy + o] = Elt<T>::from_f(acc);
}

template <typename T>
__global__ void __launch_bounds__(256) convt_direct_dgrad(const T* __restrict__ dy, const float* __restrict__ we,
                                                          T* __restrict__ dx, CtArgs a) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  const long tot = (long)a.N * a.Hi * a.Wi * a.ldx;
  if (e >= tot) return;
  const int i = (int)(e % a.ldx);
  const long p = e / a.ldx;
  if (i >= a.Ci) {
    dx[e] = Elt<T>::from_f(0.f);
    return;
  }
  const int iw = (int)(p % a.Wi), ih = (int)((p / a.Wi) % a.Hi);
  const long n = p / ((long)a.Wi * a.Hi);
  float acc = 0.f;
  for (int r = 0; r < a.K; ++r) {
    const int oh = ih * a.S - a.P + r;
    if (oh < 0 || oh >= a.Ho) continue;
    for (int s = 0; s < a.K; ++s) {
      const int ow = iw * a.S - a.P + s;
      if (ow < 0 || ow >= a.Wo) continue;
      const T* gp = dy + ((n * a.Ho + oh) * a.Wo + ow) * a.ldy;
      const float* wp = we + (long)i * a.Co * a.K * a.K + r * a.K + s;
      for (int o = 0; o < a.Co; ++o) acc = fmaf(ldv(gp + o), wp[(long)o * a.K * a.K], acc);
    }
  }
  dx[e] = Elt<T>::from_f(acc);
}

// block per (o, r, s, 16-wide input-channel chunk): G[i][o][r][s] over the block's chunk
template <typename T>
__global__ void __launch_bounds__(256) convt_direct_wgrad(const T* __restrict__ x, const T* __restrict__ dy,
                                                          float* g, CtArgs a) {
  const int nck = (a.Ci + 15) / 16;
  int b = blockIdx.x;
  const int ck = b % nck;
  b /= nck;
  const int s = b % a.K, r = (b / a.K) % a.K, o = b / (a.K * a.K);
  const int i0 = ck * 16;
  float acc[16];
#pragma unroll
  for (int j = 0; j < 16; ++j) acc[j] = 0.f;
  const long Pin = (long)a.N * a.Hi * a.Wi;
  for (long p = threadIdx.x; p < Pin; p += 256) {
    const int iw = (int)(p % a.Wi), ih = (int)((p / a.Wi) % a.Hi);
    const long n = p / ((long)a.Wi * a.Hi);
    const int oh = ih * a.S - a.P + r, ow = iw * a.S - a.P + s;
    if (oh < 0 || oh >= a.Ho || ow < 0 || ow >= a.Wo) continue;
    const float gv = ldv(dy + ((n * a.Ho + oh) * a.Wo + ow) * a.ldy + o);
    const T* xp = x + p * a.ldx + i0;
#pragma unroll
    for (int j = 0; j < 16; ++j)
      if (i0 + j < a.Ci) acc[j] = fmaf(ldv(xp + j), gv, acc[j]);
  }
  __shared__ float red[4][16];
#pragma unroll
  for (int j = 0; j < 16; ++j) {
    const float t = wave_sum(acc[j]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][j] = t;
  }
  __syncthreads();
  if (threadIdx.x < 16 && i0 + threadIdx.x < a.Ci) {
    const int i = i0 + threadIdx.x;
    g[(((long)i * a.Co + o) * a.K + r) * a.K + s] =
        red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
  }
}

// db[o] = sum over output pixels of dy[.][o]; block per o
template <typename T>
__global__ void __launch_bounds__(256) chan_sum_kernel(const T* __restrict__ dy, long P, int ld, float* db) {
  const int o = blockIdx.x;
  float s = 0.f;
  for (long p = threadIdx.x; p < P; p += 256) s += ldv(dy + p * ld + o);
  s = wave_sum(s);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) db[o] = red[0] + red[1] + red[2] + red[3];
}

// y[n][p][c] = x[n][p][c] * sa[n][c] + sb[n][c]  (sb may be null), c < C of stride ld
template <typename T>
__global__ void __launch_bounds__(256) chan_scale_fwd(const T* __restrict__ x, const float* __restrict__ sa,
                                                      const float* sb, T* __restrict__ y, long HW, int C, int ld,
                                                      long tot) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;
  if (e >= tot) return;
  const int c = (int)(e % ld);
  const long n = e / (HW * ld);
  if (c >= C) {
    y[e] = Elt<T>::from_f(0.f);
    return;
  }
  y[e] = Elt<T>::from_f(ldv(x + e) * sa[n * C + c] + (sb ? sb[n * C + c] : 0.f));
}
// backward: dx = g * sa; per (n, c): da = sum_p g x, db = sum_p g.  Block per (n, 64-channel group)
template <typename T>
__global__ void __launch_bounds__(256) chan_scale_bwd(const T* __restrict__ g, const T* __restrict__ x,
                                                      const float* __restrict__ sa, T* dx, float* da, float* db,
                                                      long HW, int C, int ld) {
  const int ngr = (C + 63) / 64;
  const int n = blockIdx.x / ngr, c = (blockIdx.x % ngr) * 64 + (threadIdx.x & 63);
  const int r = threadIdx.x >> 6;
  float s1 = 0.f, s0 = 0.f;
  if (c < C) {
    const float a = sa[(long)n * C + c];
    for (long p = r; p < HW; p += 4) {
      const long e = ((long)n * HW + p) * ld + c;
      const float gv = ldv(g + e);
      if (dx) dx[e] = Elt<T>::from_f(gv * a);
      s1 += gv * ldv(x + e);
      s0 += gv;
    }
  }
  __shared__ float red[2][4][64];
  red[0][r][threadIdx.x & 63] = s1;
  red[1][r][threadIdx.x & 63] = s0;
  __syncthreads();
  if (r == 0 && c < C) {
    const int l = threadIdx.x & 63;
    if (da) da[(long)n * C + c] = (red[0][0][l] + red[0][1][l]) + (red[0][2][l] + red[0][3][l]);
    if (db) db[(long)n * C + c] = (red[1][0][l] + red[1][1][l]) + (red[1][2][l] + red[1][3][l]);
  }
}

CtArgs make_ct(int n, int hi, int wi, int ci, int ldx, int co, int ldy, int k, int s, int p) {
  CtArgs a{};
  a.N = n; a.Hi = hi; a.Wi = wi; a.Ci = ci; a.ldx = ldx; a.Co = co; a.ldy = ldy; a.K = k; a.S = s; a.P = p;
  a.Ho = (hi - 1) * s - 2 * p + k;
  a.Wo = (wi - 1) * s - 2 * p + k;
  return a;
}

}  // namespace

extern "C" {

int fv_convt_eff_weight(const float* w, int cin, int cout, int k, int demod, float gain, float* inv, float* we,
                        void* stream) {
  FV_REQUIRE(w && we && cin > 0 && cout > 0 && k > 0 && (!demod || inv), "convt_eff_weight: bad argument");
  hipStream_t s = (hipStream_t)stream;
  int st;
  if (demod) {
    hipLaunchKernelGGL(convt_norm_any_kernel, dim3(cout), dim3(64), 0, s, w, cin, cout, k * k, inv);
    if ((st = fv_check_launch("convt_norm_any"))) return st;
  }
  const long n = (long)cin * cout * k * k;
  hipLaunchKernelGGL(convt_eff_weight_kernel, dim3(fv_cdiv(n, 256)), dim3(256), 0, s, w, demod ? inv : nullptr, gain,
                     cout, k * k, n, we);
  return fv_check_launch("convt_eff_weight");
}

int fv_convt_weight_grad(const float* w, int cin, int cout, int k, int demod, float gain, const float* inv, float* g,
                         void* stream) {
  FV_REQUIRE(w && g && (!demod || inv), "convt_weight_grad: bad argument");
  hipLaunchKernelGGL(convt_weight_grad_kernel, dim3(cout), dim3(64), 0, (hipStream_t)stream, w, demod ? inv : nullptr,
                     gain, g, cin, cout, k * k);
  return fv_check_launch("convt_weight_grad");
}

/* out [n][ho][wo][ldy] (channels >= cout written 0 only through the caller's buffer init) */
int fv_convt_direct_fwd(int dtype, const void* x, int n, int hi, int wi, int cin, int ldx, const float* we,
                        const float* bias, int cout, int ldy, int k, int stride, int pad, void* y, void* stream) {
  FV_REQUIRE(x && we && y && n > 0 && hi > 0 && wi > 0 && cin > 0 && cout > 0 && ldx >= cin && ldy >= cout,
             "convt_direct_fwd: bad argument");
  const CtArgs a = make_ct(n, hi, wi, cin, ldx, cout, ldy, k, stride, pad);
  FV_REQUIRE(a.Ho > 0 && a.Wo > 0, "convt_direct_fwd: empty output");
  const long tot = (long)n * a.Ho * a.Wo * cout;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(convt_direct_fwd<bf16>, dim3(fv_cdiv(tot, 256)), dim3(256), 0, s, (const bf16*)x, we, bias,
                       (bf16*)y, a);
  else
    hipLaunchKernelGGL(convt_direct_fwd<float>, dim3(fv_cdiv(tot, 256)), dim3(256), 0, s, (const float*)x, we, bias,
                       (float*)y, a);
  return fv_check_launch("convt_direct_fwd");
}

/* dx [n][hi][wi][ldx] (padded channels written 0) */
int fv_convt_direct_dgrad(int dtype, const void* dy, int n, int hi, int wi, int cin, int ldx, const float* we,
                          int cout, int ldy, int k, int stride, int pad, void* dx, void* stream) {
  FV_REQUIRE(dy && we && dx, "convt_direct_dgrad: null pointer");
  const CtArgs a = make_ct(n, hi, wi, cin, ldx, cout, ldy, k, stride, pad);
  const long tot = (long)n * hi * wi * ldx;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(convt_direct_dgrad<bf16>, dim3(fv_cdiv(tot, 256)), dim3(256), 0, s, (const bf16*)dy, we,
                       (bf16*)dx, a);
  else
    hipLaunchKernelGGL(convt_direct_dgrad<float>, dim3(fv_cdiv(tot, 256)), dim3(256), 0, s, (const float*)dy, we,
                       (float*)dx, a);
  return fv_check_launch("convt_direct_dgrad");
}

/* g [cin][cout][k][k] = dL/dW_eff and db [cout] (may be NULL) */
int fv_convt_direct_wgrad(int dtype, const void* x, const void* dy, int n, int hi, int wi, int cin, int ldx, int cout,
                          int ldy, int k, int stride, int pad, float* g, float* db, void* stream) {
  FV_REQUIRE(x && dy && g, "convt_direct_wgrad: null pointer");
  const CtArgs a = make_ct(n, hi, wi, cin, ldx, cout, ldy, k, stride, pad);
  hipStream_t s = (hipStream_t)stream;
  const int nb = cout * k * k * ((cin + 15) / 16);
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(convt_direct_wgrad<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)x, (const bf16*)dy, g, a);
  else
    hipLaunchKernelGGL(convt_direct_wgrad<float>, dim3(nb), dim3(256), 0, s, (const float*)x, (const float*)dy, g, a);
  int st = fv_check_launch("convt_direct_wgrad");
  if (st || !db) return st;
  const long P = (long)n * a.Ho * a.Wo;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(chan_sum_kernel<bf16>, dim3(cout), dim3(256), 0, s, (const bf16*)dy, P, ldy, db);
  else
    hipLaunchKernelGGL(chan_sum_kernel<float>, dim3(cout), dim3(256), 0, s, (const float*)dy, P, ldy, db);
  return fv_check_launch("convt_bias_grad");
}

int fv_chan_scale_fwd(int dtype, const void* x, int n, long hw, int c, int ld, const float* sa, const float* sb,
                      void* y, void* stream) {
  FV_REQUIRE(x && sa && y && n > 0 && hw > 0 && c > 0 && ld >= c, "chan_scale: bad argument");
  const long tot = (long)n * hw * ld;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(chan_scale_fwd<bf16>, dim3(fv_cdiv(tot, 256)), dim3(256), 0, s, (const bf16*)x, sa, sb, (bf16*)y,
                       hw, c, ld, tot);
  else
    hipLaunchKernelGGL(chan_scale_fwd<float>, dim3(fv_cdiv(tot, 256)), dim3(256), 0, s, (const float*)x, sa, sb,
                       (float*)y, hw, c, ld, tot);
  return fv_check_launch("chan_scale_fwd");
}

int fv_chan_scale_bwd(int dtype, const void* g, const void* x, int n, long hw, int c, int ld, const float* sa, void* dx,
                      float* da, float* db, void* stream) {
  FV_REQUIRE(g && x && sa && n > 0 && hw > 0 && c > 0 && ld >= c, "chan_scale_bwd: bad argument");
  const int nb = n * ((c + 63) / 64);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(chan_scale_bwd<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)g, (const bf16*)x, sa, (bf16*)dx,
                       da, db, hw, c, ld);
  else
    hipLaunchKernelGGL(chan_scale_bwd<float>, dim3(nb), dim3(256), 0, s, (const float*)g, (const float*)x, sa,
                       (float*)dx, da, db, hw, c, ld);
  return fv_check_launch("chan_scale_bwd");
}

}  // extern "C"
