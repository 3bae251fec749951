// Training/eval BatchNorm (nn.SyncBatchNorm, modules.py:19) split into HBM-streaming
// passes around the conv kernels:
//   stats    : per-channel (count, sum, sum of squares) in fp64, from the conv epilogue's
//              per-block partials or by streaming an NHWC tensor;  SyncBN all-reduces the
//              [3][C] record between `stats` and `finalize`.
//   finalize : mean / invstd, fused affine (scale, shift), running stats (momentum 0.1,
//              unbiased variance) -> torch/nn/modules/_functions.py:10-125 semantics.
//   act fwd  : out = [avgpool2](act(y*scale + shift))  (CNA + DownBlock2D's AvgPool2d).
//   bwd      : g = dout * act'(.)  ->  sums (g, g*yhat)  ->  dx = gamma*invstd*(g - k0 - yhat*k1)
#include "common.h"

namespace {

constexpr int NSPLIT = 128;   // level-1 splits of the conv-partials reduction
constexpr int MAXBLK = 1024;  // max blocks (= level-1 records) of the streaming reductions
constexpr int NTH = 256;

// blocks of a streaming per-channel reduction over `pixels` x (C/8) chunks: >= 8 chunks per thread
int stream_blocks(long pixels, int C) {
  const long work = pixels * (C / 8);
  long b = (work + NTH * 8 - 1) / (NTH * 8);
  if (b < 1) b = 1;
  if (b > MAXBLK) b = MAXBLK;
  return (int)b;
}

template <typename T>
__device__ __forceinline__ void ld8(const T* p, float* f) {
  Chunk8<T> c;
  c.load(p);
#pragma unroll
  for (int j = 0; j < 8; ++j) f[j] = c.get(j);
}
template <typename T>
__device__ __forceinline__ void st8(T* p, const float* f) {
  Chunk8<T> c;
  c.set8(f);
  c.store(p);
}

// conv per-block (sum, centred M2) partials -> ws [split][3][C] (n, S, Q) in fp64
__global__ void partials_kernel(const float* __restrict__ part, int nb, int bpix, long P, int C,
                                double* ws) {
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int r = threadIdx.x >> 6;
  const int split = blockIdx.y;
  const int per = (nb + NSPLIT - 1) / NSPLIT;
  const int b0 = split * per, b1 = min(nb, b0 + per);
  double n = 0, S = 0, Q = 0;
  if (c < C) {
    for (int b = b0 + r; b < b1; b += 4) {
      const double nb_ = (double)min((long)bpix, P - (long)b * bpix);
      const double s = part[(long)(2 * b) * C + c], m2 = part[(long)(2 * b + 1) * C + c];
      n += nb_;
      S += s;
      Q += m2 + s * s / nb_;
    }
  }
  __shared__ double red[3][4][64];
  red[0][r][threadIdx.x & 63] = n;
  red[1][r][threadIdx.x & 63] = S;
  red[2][r][threadIdx.x & 63] = Q;
  __syncthreads();
  if (r == 0 && c < C) {
    for (int j = 0; j < 3; ++j) {
      double t = 0;
      for (int k = 0; k < 4; ++k) t += red[j][k][threadIdx.x];
      ws[((long)split * 3 + j) * C + c] = t;
    }
  }
}

// streaming statistics of x [P][ldc] -> ws [block][3][C]; thread = (pixel row, 8-channel group)
template <typename T>
__global__ void tensor_stats_kernel(const T* __restrict__ x, long P, int C, int ldc, double* ws) {
  const int tpp = C / 8;                 // threads per pixel (NTH % tpp == 0)
  const int rows = NTH / tpp;
  const int cg = threadIdx.x % tpp, row = threadIdx.x / tpp;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  long cnt = 0;
  for (long p = (long)blockIdx.x * rows + row; p < P; p += (long)gridDim.x * rows) {
    float f[8];
    ld8<T>(x + p * ldc + cg * 8, f);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += f[j];
      q[j] += f[j] * f[j];
    }
    ++cnt;
  }
  __shared__ float ss[2][NTH * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss[0][row * C + cg * 8 + j] = s[j];
    ss[1][row * C + cg * 8 + j] = q[j];
  }
  __shared__ long cn[NTH];
  cn[threadIdx.x] = cnt;
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NTH) {
    double a = 0, b = 0;
    long n = 0;
    for (int r = 0; r < rows; ++r) {
      a += ss[0][r * C + c];
      b += ss[1][r * C + c];
      n += cn[r * tpp];
    }
    ws[((long)blockIdx.x * 3 + 0) * C + c] = (double)n;
    ws[((long)blockIdx.x * 3 + 1) * C + c] = a;
    ws[((long)blockIdx.x * 3 + 2) * C + c] = b;
  }
}

// out[i] = sum_s ws[s][i], i < rec*C : one wave per output (lanes stride the splits), 4 per block
__global__ void sum_splits_kernel(const double* ws, int nsplit, int rec, int C, double* out) {
  const int n = rec * C;
  const int i = blockIdx.x * 4 + (threadIdx.x >> 6);
  const int lane = threadIdx.x & 63;
  if (i >= n) return;
  double t0 = 0, t1 = 0, t2 = 0, t3 = 0;
  int s = lane;
  for (; s + 192 < nsplit; s += 256) {
    t0 += ws[(long)s * n + i];
    t1 += ws[(long)(s + 64) * n + i];
    t2 += ws[(long)(s + 128) * n + i];
    t3 += ws[(long)(s + 192) * n + i];
  }
  for (; s < nsplit; s += 64) t0 += ws[(long)s * n + i];
  const double t = wave_sum_d((t0 + t1) + (t2 + t3));
  if (lane == 0) out[i] = t;
}

__global__ void finalize_kernel(const double* stats, int C, const float* gamma, const float* beta,
                                float eps, float mom, int training, float* rm, float* rv,
                                float* save_mean, float* save_invstd, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  double mean, var;
  if (training) {
    const double n = stats[c], S = stats[C + c], Q = stats[2 * C + c];
    mean = S / n;
    var = Q / n - mean * mean;
    if (var < 0) var = 0;
    if (rm) rm[c] = (float)((1.0 - mom) * rm[c] + mom * mean);
    if (rv) rv[c] = (float)((1.0 - mom) * rv[c] + mom * (n > 1 ? var * n / (n - 1) : var));
  } else {
    mean = rm[c];
    var = rv[c];
  }
  const float inv = (float)(1.0 / sqrt(var + (double)eps));
  const float g = gamma ? gamma[c] : 1.f, b = beta ? beta[c] : 0.f;
  if (save_mean) save_mean[c] = (float)mean;
  if (save_invstd) save_invstd[c] = inv;
  const float sc = g * inv;
  if (scale) scale[c] = sc;
  if (shift) shift[c] = b - (float)mean * sc;
}

// out = [pool](act(y*scale+shift)); one thread per (out pixel, 8-channel chunk)
template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ y, int N, int H, int W, int C, int ldc,
                               const float* __restrict__ scale, const float* __restrict__ shift,
                               float slope, int pool, T* out) {
  const int cpc = C / 8;
  const int Ho = pool ? H / 2 : H, Wo = pool ? W / 2 : W;
  const long total = (long)N * Ho * Wo * cpc;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(e % cpc);
    const long po = e / cpc;
    const int c = cg * 8;
    float sc[8], sh[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) { sc[j] = scale[c + j]; sh[j] = shift[c + j]; }
    float o[8];
    if (!pool) {
      float f[8];
      ld8<T>(y + po * ldc + c, f);
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = fv_act(f[j] * sc[j] + sh[j], slope);
    } else {
      const int n = (int)(po / (Ho * Wo));
      const int rem = (int)(po - (long)n * Ho * Wo);
      const int i = rem / Wo, jx = rem - i * Wo;
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] = 0.f;
#pragma unroll
      for (int dy = 0; dy < 2; ++dy)
#pragma unroll
        for (int dx = 0; dx < 2; ++dx) {
          float f[8];
          ld8<T>(y + ((long)(n * H + 2 * i + dy) * W + 2 * jx + dx) * ldc + c, f);
#pragma unroll
          for (int j = 0; j < 8; ++j) o[j] += fv_act(f[j] * sc[j] + sh[j], slope);
        }
#pragma unroll
      for (int j = 0; j < 8; ++j) o[j] *= 0.25f;
    }
    st8<T>(out + po * C + c, o);
  }
}

// g at a full-resolution pixel (n,h,w), 8 channels; pooled dout is [N][H/2][W/2][C]
template <typename T>
__device__ __forceinline__ void grad_g(const T* dout, const T* y, long p, int n, int h, int w, int H,
                                       int W, int C, int ldc, int c, int pool, const float* mean,
                                       const float* invstd, const float* gamma, const float* beta,
                                       float slope, float* g, float* yh) {
  float d[8], v[8];
  if (pool) {
    ld8<T>(dout + ((long)(n * (H / 2) + h / 2) * (W / 2) + w / 2) * C + c, d);
#pragma unroll
    for (int j = 0; j < 8; ++j) d[j] *= 0.25f;
  } else {
    ld8<T>(dout + p * ldc + c, d);
  }
  ld8<T>(y + p * ldc + c, v);
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    yh[j] = (v[j] - mean[c + j]) * invstd[c + j];
    const float z = gamma[c + j] * yh[j] + beta[c + j];
    g[j] = z > 0.f ? d[j] : d[j] * slope;
  }
}

template <typename T>
__global__ void act_bwd_reduce_kernel(const T* __restrict__ dout, const T* __restrict__ y, int N, int H,
                                      int W, int C, int ldc, const float* mean, const float* invstd,
                                      const float* gamma, const float* beta, float slope, int pool,
                                      double* ws) {
  const int tpp = C / 8;
  const int rows = NTH / tpp;
  const int cg = threadIdx.x % tpp, row = threadIdx.x / tpp;
  const long P = (long)N * H * W;
  float s[8], q[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q[j] = 0.f;
  for (long p = (long)blockIdx.x * rows + row; p < P; p += (long)gridDim.x * rows) {
    const int n = (int)(p / ((long)H * W));
    const int rem = (int)(p - (long)n * H * W);
    const int h = rem / W, w = rem - h * W;
    float g[8], yh[8];
    grad_g<T>(dout, y, p, n, h, w, H, W, C, ldc, cg * 8, pool, mean, invstd, gamma, beta, slope, g, yh);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += g[j];
      q[j] += g[j] * yh[j];
    }
  }
  __shared__ float ss[2][NTH * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss[0][row * C + cg * 8 + j] = s[j];
    ss[1][row * C + cg * 8 + j] = q[j];
  }
  __syncthreads();
  for (int c = threadIdx.x; c < C; c += NTH) {
    double a = 0, b = 0;
    for (int r = 0; r < rows; ++r) {
      a += ss[0][r * C + c];
      b += ss[1][r * C + c];
    }
    ws[((long)blockIdx.x * 2 + 0) * C + c] = a;
    ws[((long)blockIdx.x * 2 + 1) * C + c] = b;
  }
}

__global__ void bwd_finalize_kernel(const double* red, int C, double count, float* dgamma, float* dbeta,
                                    float* k) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double sg = red[c], sgy = red[C + c];
  if (dbeta) dbeta[c] = (float)sg;
  if (dgamma) dgamma[c] = (float)sgy;
  k[c] = (float)(sg / count);
  k[C + c] = (float)(sgy / count);
}

template <typename T>
__global__ void act_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ y, int N, int H,
                                     int W, int C, int ldc, const float* mean, const float* invstd,
                                     const float* gamma, const float* beta, float slope, int pool,
                                     const float* __restrict__ k, const T* addend, T* dx) {
  const int cpc = C / 8;
  const long total = (long)N * H * W * cpc;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int cg = (int)(e % cpc);
    const long p = e / cpc;
    const int c = cg * 8;
    const int n = (int)(p / ((long)H * W));
    const int rem = (int)(p - (long)n * H * W);
    const int h = rem / W, w = rem - h * W;
    float g[8], yh[8], o[8];
    grad_g<T>(dout, y, p, n, h, w, H, W, C, ldc, c, pool, mean, invstd, gamma, beta, slope, g, yh);
    float ad[8];
    if (addend) ld8<T>(addend + p * ldc + c, ad);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      o[j] = gamma[c + j] * invstd[c + j] * (g[j] - k[c + j] - yh[j] * k[C + c + j]);
      if (addend) o[j] += ad[j];
    }
    st8<T>(dx + p * ldc + c, o);
  }
}

int grid_for(long work, int cap = 8192) {
  long g = (work + NTH - 1) / NTH;
  if (g < 1) g = 1;
  if (g > cap) g = cap;
  return (int)g;
}

int check_c(int c, int ldc) {
  FV_REQUIRE(c > 0 && c % 8 == 0 && c <= 8 * NTH && NTH % (c / 8) == 0,
             "bn: channels must be 8 * a power of two <= 2048 (got %d)", c);
  FV_REQUIRE(ldc >= c && ldc % 8 == 0, "bn: bad channel stride %d", ldc);
  return FV_OK;
}

}  // namespace

extern "C" {

size_t fv_bn_ws_bytes(int c) { return (size_t)MAXBLK * 3 * c * sizeof(double); }

int fv_bn_stats_from_partials(const float* partials, int nblocks, int block_pixels, long total_pixels,
                              int c, double* stats, void* ws, void* stream) {
  FV_REQUIRE(partials && stats && ws, "null pointer");
  FV_REQUIRE(nblocks > 0 && c > 0, "bad sizes");
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(partials_kernel, dim3(fv_cdiv(c, 64), NSPLIT), dim3(NTH), 0, s, partials, nblocks,
                     block_pixels, total_pixels, c, (double*)ws);
  int st = fv_check_launch("bn_partials");
  if (st) return st;
  hipLaunchKernelGGL(sum_splits_kernel, dim3(fv_cdiv(3 * c, 4)), dim3(NTH), 0, s, (const double*)ws, NSPLIT,
                     3, c, stats);
  return fv_check_launch("bn_sum_splits");
}

int fv_bn_stats_tensor(int dtype, const void* x, long pixels, int c, int ldc, double* stats, void* ws,
                       void* stream) {
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(x && stats && ws, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int nb = stream_blocks(pixels, c);
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(tensor_stats_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)x, pixels, c, ldc,
                       (double*)ws);
  else
    hipLaunchKernelGGL(tensor_stats_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)x, pixels, c, ldc,
                       (double*)ws);
  if ((st = fv_check_launch("bn_tensor_stats"))) return st;
  hipLaunchKernelGGL(sum_splits_kernel, dim3(fv_cdiv(3 * c, 4)), dim3(NTH), 0, s, (const double*)ws, nb, 3, c,
                     stats);
  return fv_check_launch("bn_sum_splits");
}

int fv_bn_finalize(const double* stats, int c, const float* gamma, const float* beta, float eps,
                   float momentum, int training, float* running_mean, float* running_var, float* save_mean,
                   float* save_invstd, float* scale, float* shift, void* stream) {
  FV_REQUIRE(c > 0, "bad channels");
  FV_REQUIRE(!training || stats, "training finalize needs stats");
  FV_REQUIRE(training || (running_mean && running_var), "eval finalize needs running stats");
  hipLaunchKernelGGL(finalize_kernel, dim3(fv_cdiv(c, NTH)), dim3(NTH), 0, (hipStream_t)stream, stats, c, gamma,
                     beta, eps, momentum, training, running_mean, running_var, save_mean, save_invstd, scale,
                     shift);
  return fv_check_launch("bn_finalize");
}

int fv_bn_act_fwd(int dtype, const void* y, int n, int h, int w, int c, int ldc, const float* scale,
                  const float* shift, float slope, int pool, void* out, void* stream) {
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(!pool || (h % 2 == 0 && w % 2 == 0), "pool needs even h, w");
  const long work = (long)n * (pool ? h / 2 : h) * (pool ? w / 2 : w) * (c / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(act_fwd_kernel<bf16>, dim3(grid_for(work)), dim3(NTH), 0, s, (const bf16*)y, n, h, w, c,
                       ldc, scale, shift, slope, pool, (bf16*)out);
  else
    hipLaunchKernelGGL(act_fwd_kernel<float>, dim3(grid_for(work)), dim3(NTH), 0, s, (const float*)y, n, h, w, c,
                       ldc, scale, shift, slope, pool, (float*)out);
  return fv_check_launch("bn_act_fwd");
}

int fv_bn_act_bwd_reduce(int dtype, const void* dout, const void* y, int n, int h, int w, int c, int ldc,
                         const float* mean, const float* invstd, const float* gamma, const float* beta,
                         float slope, int pool, double* red, void* ws, void* stream) {
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(!pool || ldc == c, "pooled bwd needs dense channels");
  hipStream_t s = (hipStream_t)stream;
  const int nb = stream_blocks((long)n * h * w, c);
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(act_bwd_reduce_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)dout,
                       (const bf16*)y, n, h, w, c, ldc, mean, invstd, gamma, beta, slope, pool, (double*)ws);
  else
    hipLaunchKernelGGL(act_bwd_reduce_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)dout,
                       (const float*)y, n, h, w, c, ldc, mean, invstd, gamma, beta, slope, pool, (double*)ws);
  if ((st = fv_check_launch("bn_bwd_reduce"))) return st;
  hipLaunchKernelGGL(sum_splits_kernel, dim3(fv_cdiv(2 * c, 4)), dim3(NTH), 0, s, (const double*)ws, nb, 2, c,
                     red);
  return fv_check_launch("bn_sum_splits");
}

int fv_bn_bwd_finalize(const double* red, int c, long count, float* dgamma, float* dbeta, float* k,
                       void* stream) {
  FV_REQUIRE(red && k && count > 0, "bad args");
  hipLaunchKernelGGL(bwd_finalize_kernel, dim3(fv_cdiv(c, NTH)), dim3(NTH), 0, (hipStream_t)stream, red, c,
                     (double)count, dgamma, dbeta, k);
  return fv_check_launch("bn_bwd_finalize");
}

int fv_bn_act_bwd_apply(int dtype, const void* dout, const void* y, int n, int h, int w, int c, int ldc,
                        const float* mean, const float* invstd, const float* gamma, const float* beta,
                        float slope, int pool, const float* k, const void* addend, void* dx, void* stream) {
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(!pool || ldc == c, "pooled bwd needs dense channels");
  const long work = (long)n * h * w * (c / 8);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(act_bwd_apply_kernel<bf16>, dim3(grid_for(work)), dim3(NTH), 0, s, (const bf16*)dout,
                       (const bf16*)y, n, h, w, c, ldc, mean, invstd, gamma, beta, slope, pool, k,
                       (const bf16*)addend, (bf16*)dx);
  else
    hipLaunchKernelGGL(act_bwd_apply_kernel<float>, dim3(grid_for(work)), dim3(NTH), 0, s, (const float*)dout,
                       (const float*)y, n, h, w, c, ldc, mean, invstd, gamma, beta, slope, pool, k,
                       (const float*)addend, (float*)dx);
  return fv_check_launch("bn_bwd_apply");
}

}  // extern "C"
