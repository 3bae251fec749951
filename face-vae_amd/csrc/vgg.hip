// Elementwise / pooling kernels of the perceptual loss (losses.py:33-151) for gfx950: the VGG
// feature stacks run their 3x3 convs on conv.hip; what remains is HBM-bound NHWC passes.
//   relu_bwd      nn.ReLU backward (mask from the stored output)
//   maxpool2      nn.MaxPool2d(2, 2) forward / backward (argmax recomputed; the first maximum
//                 in (kh, kw) order wins, as torch)
//   avgpool2_bwd  adjoint of the 2x2 average (== F.interpolate(scale 0.5, bilinear,
//                 align_corners=False) on even sizes, losses.py:148-149)
//   l1            nn.L1Loss mean |a - b| (deterministic two-level sum) and its gradient
#include <algorithm>

#include "common.h"

namespace {

__device__ __forceinline__ float ldf(const float* p) { return *p; }
__device__ __forceinline__ float ldf(const bf16* p) { return (float)*p; }

template <typename T>
__global__ void __launch_bounds__(256) relu_bwd_kernel(const T* __restrict__ g, const T* __restrict__ y,
                                                       T* __restrict__ dx, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) dx[i] = ldf(y + i) > 0.f ? g[i] : Elt<T>::from_f(0.f);
}

// x [N][H][W][C] -> y [N][H/2][W/2][C]; one thread per output element
template <typename T>
__global__ void __launch_bounds__(256) maxpool2_fwd_kernel(const T* __restrict__ x, T* __restrict__ y, int N, int H,
                                                           int W, int C) {
  const int Ho = H / 2, Wo = W / 2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * Ho * Wo * C) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int wo = (int)(p % Wo), ho = (int)((p / Wo) % Ho);
  const long n = p / ((long)Wo * Ho);
  const T* b = x + ((n * H + 2 * ho) * W + 2 * wo) * C + c;
  float m = ldf(b);
  m = fmaxf(m, ldf(b + C));
  m = fmaxf(m, ldf(b + (long)W * C));
  m = fmaxf(m, ldf(b + (long)W * C + C));
  y[i] = Elt<T>::from_f(m);
}

// dx (fully written): the output gradient goes to the window's first maximum
template <typename T>
__global__ void __launch_bounds__(256) maxpool2_bwd_kernel(const T* __restrict__ x, const T* __restrict__ g,
                                                           T* __restrict__ dx, int N, int H, int W, int C) {
  const int Ho = H / 2, Wo = W / 2;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * Ho * Wo * C) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int wo = (int)(p % Wo), ho = (int)((p / Wo) % Ho);
  const long n = p / ((long)Wo * Ho);
  const long o[4] = {0, C, (long)W * C, (long)W * C + C};
  const long base = ((n * H + 2 * ho) * W + 2 * wo) * C + c;
  float m = ldf(x + base);
  int am = 0;
#pragma unroll
  for (int k = 1; k < 4; ++k) {
    const float v = ldf(x + base + o[k]);
    if (v > m) {
      m = v;
      am = k;
    }
  }
  const float gv = ldf(g + i);
#pragma unroll
  for (int k = 0; k < 4; ++k) dx[base + o[k]] = Elt<T>::from_f(k == am ? gv : 0.f);
}

// dx[n][h][w][c] = g[n][h/2][w/2][c] / 4
template <typename T>
__global__ void __launch_bounds__(256) avgpool2_bwd_kernel(const T* __restrict__ g, T* __restrict__ dx, int N, int H,
                                                           int W, int C) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * H * W * C) return;
  const int c = (int)(i % C);
  const long p = i / C;
  const int w = (int)(p % W), h = (int)((p / W) % H);
  const long n = p / ((long)W * H);
  dx[i] = Elt<T>::from_f(0.25f * ldf(g + ((n * (H / 2) + h / 2) * (W / 2) + w / 2) * C + c));
}

constexpr int L1_BLOCKS = 1024;
template <typename T>
__global__ void __launch_bounds__(256) l1_partial_kernel(const T* __restrict__ a, const T* __restrict__ b, long n,
                                                         double* part) {
  double s = 0.0;
  for (long i = (long)blockIdx.x * 256 + threadIdx.x; i < n; i += (long)gridDim.x * 256)
    s += (double)fabsf(ldf(a + i) - ldf(b + i));
  s = wave_sum_d(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) part[blockIdx.x] = red[0] + red[1] + red[2] + red[3];
}
__global__ void __launch_bounds__(256) l1_final_kernel(const double* __restrict__ part, int np, double inv_n,
                                                       float* out) {
  double s = 0.0;
  for (int i = threadIdx.x; i < np; i += 256) s += part[i];
  s = wave_sum_d(s);
  __shared__ double red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = s;
  __syncthreads();
  if (threadIdx.x == 0) out[0] = (float)((red[0] + red[1] + red[2] + red[3]) * inv_n);
}
// da = gout * sign(a - b) / n
template <typename T>
__global__ void __launch_bounds__(256) l1_bwd_kernel(const T* __restrict__ a, const T* __restrict__ b, long n,
                                                     const float* gout, float scale, T* __restrict__ da) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const float d = ldf(a + i) - ldf(b + i);
  const float s = d > 0.f ? 1.f : (d < 0.f ? -1.f : 0.f);
  da[i] = Elt<T>::from_f(s * gout[0] * scale);
}

}  // namespace

extern "C" {

int fv_relu_bwd(int dtype, const void* g, const void* y, long n, void* dx, void* stream) {
  FV_REQUIRE(g && y && dx && n >= 0, "relu_bwd: bad argument");
  if (n == 0) return FV_OK;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(relu_bwd_kernel<bf16>, dim3(fv_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)g,
                       (const bf16*)y, (bf16*)dx, n);
  else
    hipLaunchKernelGGL(relu_bwd_kernel<float>, dim3(fv_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, (const float*)g,
                       (const float*)y, (float*)dx, n);
  return fv_check_launch("relu_bwd");
}

int fv_maxpool2_fwd(int dtype, const void* x, int n, int h, int w, int c, void* y, void* stream) {
  FV_REQUIRE(x && y && n > 0 && h >= 2 && w >= 2 && c > 0, "maxpool2: bad argument");
  const long m = (long)n * (h / 2) * (w / 2) * c;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(maxpool2_fwd_kernel<bf16>, dim3(fv_cdiv(m, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)x, (bf16*)y, n, h, w, c);
  else
    hipLaunchKernelGGL(maxpool2_fwd_kernel<float>, dim3(fv_cdiv(m, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, (float*)y, n, h, w, c);
  return fv_check_launch("maxpool2_fwd");
}

/* dx [n][h][w][c] fully written (h, w even) */
int fv_maxpool2_bwd(int dtype, const void* x, const void* g, int n, int h, int w, int c, void* dx, void* stream) {
  FV_REQUIRE(x && g && dx && n > 0 && h % 2 == 0 && w % 2 == 0 && c > 0, "maxpool2_bwd: h, w must be even");
  const long m = (long)n * (h / 2) * (w / 2) * c;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(maxpool2_bwd_kernel<bf16>, dim3(fv_cdiv(m, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)x, (const bf16*)g, (bf16*)dx, n, h, w, c);
  else
    hipLaunchKernelGGL(maxpool2_bwd_kernel<float>, dim3(fv_cdiv(m, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)x, (const float*)g, (float*)dx, n, h, w, c);
  return fv_check_launch("maxpool2_bwd");
}

int fv_avgpool2_bwd(int dtype, const void* g, int n, int h, int w, int c, void* dx, void* stream) {
  FV_REQUIRE(g && dx && n > 0 && h % 2 == 0 && w % 2 == 0 && c > 0, "avgpool2_bwd: h, w must be even");
  const long m = (long)n * h * w * c;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(avgpool2_bwd_kernel<bf16>, dim3(fv_cdiv(m, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)g, (bf16*)dx, n, h, w, c);
  else
    hipLaunchKernelGGL(avgpool2_bwd_kernel<float>, dim3(fv_cdiv(m, 256)), dim3(256), 0, (hipStream_t)stream,
                       (const float*)g, (float*)dx, n, h, w, c);
  return fv_check_launch("avgpool2_bwd");
}

size_t fv_l1t_ws_bytes(void) { return L1_BLOCKS * sizeof(double); }

/* loss[0] = mean |a - b| over n elements (bf16 or f32 operands) */
int fv_l1t_fwd(int dtype, const void* a, const void* b, long n, float* loss, void* ws, void* stream) {
  FV_REQUIRE(a && b && loss && ws && n > 0, "l1t: bad argument");
  const int nb = (int)std::min<long>(L1_BLOCKS, fv_cdiv(n, 256));
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(l1_partial_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)a, (const bf16*)b, n, (double*)ws);
  else
    hipLaunchKernelGGL(l1_partial_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)a, (const float*)b, n,
                       (double*)ws);
  int st = fv_check_launch("l1t_partial");
  if (st) return st;
  hipLaunchKernelGGL(l1_final_kernel, dim3(1), dim3(256), 0, s, (const double*)ws, nb, 1.0 / (double)n, loss);
  return fv_check_launch("l1t_final");
}

/* da = gout[0] * scale * sign(a - b)   (scale = 1 / n for the mean) */
int fv_l1t_bwd(int dtype, const void* a, const void* b, long n, const float* gout, float scale, void* da,
               void* stream) {
  FV_REQUIRE(a && b && gout && da && n > 0, "l1t_bwd: bad argument");
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(l1_bwd_kernel<bf16>, dim3(fv_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, (const bf16*)a,
                       (const bf16*)b, n, gout, scale, (bf16*)da);
  else
    hipLaunchKernelGGL(l1_bwd_kernel<float>, dim3(fv_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, (const float*)a,
                       (const float*)b, n, gout, scale, (float*)da);
  return fv_check_launch("l1t_bwd");
}

}  // extern "C"
