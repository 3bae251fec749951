// Training/eval BatchNorm (nn.SyncBatchNorm, modules.py:19) split into HBM-streaming
// passes around the conv kernels:
//   stats    : per-channel (count, sum, sum of squares) in fp64, from the conv epilogue's
//              per-block partials or by streaming an NHWC tensor;  SyncBN all-reduces the
//              [3][C] record between `stats` and `finalize`.
//   finalize : mean / invstd, fused affine (scale, shift), running stats (momentum 0.1,
//              unbiased variance) -> torch/nn/modules/_functions.py:10-125 semantics.
//   act fwd  : out = [avgpool2](act(y*scale + shift))  (CNA + DownBlock2D's AvgPool2d).
//   bwd      : g = dout * act'(.)  ->  sums (g, g*yhat)  ->  dx = gamma*invstd*(g - k0 - yhat*k1)
#include <stdlib.h>

#include <atomic>

#include "common.h"

namespace {

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

// mean / invstd / fused affine / running statistics of one channel from (n, S, Q)
__device__ __forceinline__ void bn_finalize_one(int c, int C, double n, double S, double Q, const float* gamma,
                                                const float* beta, float eps, float mom, int training, float* rm,
                                                float* rv, float* save_mean, float* save_invstd, float* scale,
                                                float* shift) {
  double mean, var;
  if (training) {
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

__global__ void finalize_kernel(const double* stats, int C, const float* gamma, const float* beta,
                                float eps, float mom, int training, float* rm, float* rv, long long* nbt,
                                float* save_mean, float* save_invstd, float* scale, float* shift) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (nbt && training && c == 0) nbt[0] += 1;
  if (c >= C) return;
  const double n = training ? stats[c] : 0, S = training ? stats[C + c] : 0, Q = training ? stats[2 * C + c] : 0;
  bn_finalize_one(c, C, n, S, Q, gamma, beta, eps, mom, training, rm, rv, save_mean, save_invstd, scale, shift);
}

// ---------------------------------------------------------------------------------------------
// Record folds (+ finalize): the per-channel sums of a BN layer arrive as `nrec` rows of partial
// sums -- fp32 (sum, sum of squares) records of a conv epilogue / store pass ([r][2][C]), or the
// fp64 per-block rows of a streaming pass ([b][3][C] with a count row, [b][2][C] backward sums).
// ONE launch folds up to FOLD2 records and finishes the layer: one channel per block of 1024
// threads (fold1_kernel).  More records (the full-resolution layers' 16k conv records): chunk
// partials [chunk][NV][C] from blocks that own 8 channels and read whole 32 / 64-B channel
// octets of their rows (fold_part_kernel), into the caller's workspace, then fold1 over them
// (r3 folded 16k rows in one launch, 4 B per 128-B line: 45-70 us; now 23-25 us).  Fixed order
// (rows in thread order, a fixed xor tree per wave, waves in order, chunks in order):
// bit-reproducible.
// (measured and not kept, r4: octet blocks for every fold -- 1024-row folds 11-21 us against
// fold1's 8-13, 4096-row folds 10.6 + 3.9 us against 11.4; one launch with the chunks published by an agent-scope release + arrival
// counter, the last block adding them -- the release writes back the XCD's L2 per block: +6..8
// us per fold, step 12.50 -> 12.86 ms.)
// ---------------------------------------------------------------------------------------------
constexpr int FOLDB = 256, FOLDR = 1024;    // threads per octet fold block, records per fold block
constexpr int FOLDT = 1024;                 // threads per one-channel fold block
constexpr int FOLD2 = 8192;                 // records above which the fold takes two levels
enum { FOLD_STATS = 0, FOLD_FWD = 1, FOLD_BWD = 2 };
struct FoldArgs {
  const void* src;
  int nrec, C;
  long rstride;              // elements between rows
  long P;                    // element count per channel when the rows carry none (NV = 2 forward)
  // FOLD_STATS: the fp64 [3][C] (n, S, Q) record (the SyncBN all-reduce payload)
  double* stats;
  // FOLD_FWD: finalize (bn_finalize_one)
  const float *gamma, *beta;
  float eps, mom;
  float *rm, *rv;
  long long* nbt;
  float *save_mean, *save_invstd, *scale, *shift;
  // FOLD_BWD: dbeta = sum g, dgamma = sum g*yhat (rank-local), k = (sums) / count (count > 0),
  // red = the fp64 [2][C] sums (SyncBN payload), each optional
  double count;
  float *dgamma, *dbeta, *k;
  double* red;
};

// 8 consecutive channels of one row (T = float records / double streaming rows) into acc
template <typename T>
__device__ __forceinline__ void fold_load8(const T* p, double* acc) {
  if constexpr (sizeof(T) == 4) {
    const float4 a = reinterpret_cast<const float4*>(p)[0], b = reinterpret_cast<const float4*>(p)[1];
    acc[0] += a.x; acc[1] += a.y; acc[2] += a.z; acc[3] += a.w;
    acc[4] += b.x; acc[5] += b.y; acc[6] += b.z; acc[7] += b.w;
  } else {
#pragma unroll
    for (int h = 0; h < 4; ++h) {
      const double2 d = reinterpret_cast<const double2*>(p)[h];
      acc[2 * h] += d.x;
      acc[2 * h + 1] += d.y;
    }
  }
}

// level 1 of a fold of more than FOLDR records: block (octet, chunk) sums rows [chunk FOLDR,
// (chunk + 1) FOLDR) of 8 channels -> part [chunk][NV][C] (fp64)
template <typename T, int NV>
__global__ void __launch_bounds__(FOLDB) fold_part_kernel(FoldArgs a, double* part) {
  const int c0 = blockIdx.x * 8, ch = blockIdx.y, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int r0 = ch * FOLDR, r1 = min(a.nrec, r0 + FOLDR);
  double acc[NV][8];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int q = 0; q < 8; ++q) acc[v][q] = 0.0;
  const T* src = reinterpret_cast<const T*>(a.src) + c0;
#pragma unroll 2
  for (int r = r0 + tid; r < r1; r += FOLDB) {
    const T* p = src + (long)r * a.rstride;
#pragma unroll
    for (int v = 0; v < NV; ++v) fold_load8<T>(p + (long)v * a.C, acc[v]);
  }
  __shared__ double red[FOLDB / 64][NV * 8];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      const double t = wave_sum_d(acc[v][q]);
      if (lane == 0) red[w][v * 8 + q] = t;
    }
  __syncthreads();
  if (tid >= 8) return;
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double t = 0.0;
#pragma unroll
    for (int j = 0; j < FOLDB / 64; ++j) t += red[j][v * 8 + tid];
    part[((long)ch * NV + v) * a.C + c0 + tid] = t;
  }
}

template <int NV, int MODE>
__device__ __forceinline__ void fold_finish(const FoldArgs& a, int c, const double* tot);

// <= FOLD2 records (and level 2): one channel per block of 1024 threads, rows t, t + 1024, ...
template <typename T, int NV, int MODE>
__global__ void __launch_bounds__(FOLDT) fold1_kernel(FoldArgs a) {
  const int c = blockIdx.x, tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const T* src = reinterpret_cast<const T*>(a.src) + c;
  const long vs = a.C;
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
#pragma unroll 8
  for (int r = tid; r < a.nrec; r += FOLDT) {
    const T* p = src + (long)r * a.rstride;
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] += (double)p[v * vs];
  }
  __shared__ double red[NV][FOLDT / 64];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    const double t = wave_sum_d(acc[v]);
    if (lane == 0) red[v][w] = t;
  }
  __syncthreads();
  if (tid != 0) return;
  double tot[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double t = 0.0;
    for (int j = 0; j < FOLDT / 64; ++j) t += red[v][j];
    tot[v] = t;
  }
  fold_finish<NV, MODE>(a, c, tot);
}

// <= FOLD2 records, C % 16 == 0: one block per 16 channels, so every row is read as whole 64-B
// (fp32) / 128-B (fp64) channel segments -- fold1 reads 4 B per sector of each row (r4: 13 us
// for the 2048-record, 256-channel res-conv folds).  Lane l of a wave: channel l & 15 of row
// (l >> 4) + 4 w + 64 i; fixed reduction order (xor tree over the 4 row lanes, waves in order).
template <typename T, int NV, int MODE>
__global__ void __launch_bounds__(FOLDT) fold16_kernel(FoldArgs a) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c0 = blockIdx.x * 16, cl = lane & 15;
  const T* src = reinterpret_cast<const T*>(a.src) + c0 + cl;
  const long vs = a.C;
  double acc[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) acc[v] = 0.0;
#pragma unroll 4
  for (int r = (lane >> 4) + 4 * w; r < a.nrec; r += FOLDT / 16) {
    const T* p = src + (long)r * a.rstride;
#pragma unroll
    for (int v = 0; v < NV; ++v) acc[v] += (double)p[v * vs];
  }
  __shared__ double red[FOLDT / 64][NV][16];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double t = acc[v];
    t += __shfl_xor(t, 16, 64);
    t += __shfl_xor(t, 32, 64);
    if (lane < 16) red[w][v][lane] = t;
  }
  __syncthreads();
  if (tid >= 16) return;
  double tot[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    double t = 0.0;
    for (int j = 0; j < FOLDT / 64; ++j) t += red[j][v][tid];
    tot[v] = t;
  }
  fold_finish<NV, MODE>(a, c0 + tid, tot);
}

// level 1 of a fold of fp32 records with scratch: block (16-channel group, chunk of `rows`
// records) -> part [chunk][NV][C] (fp64).  4 lanes per record row (16 B each: a whole 64-B
// channel segment per row), 16 rows per wave load, every load of the chunk in flight at once
// (the one-launch fold16 over 16-64 blocks was latency-bound: 16 us for 2048 records).
// Level 2 in the same launch (r6): the chunk rows of a 16-channel group are stored
// write-through (sc1, no L2 write-back), wave 0 -- the only storing wave -- drains them and takes
// the group's arrival ticket (relaxed agent atomic); the group's last arriver acquires once and
// sums the chunk rows in chunk order (sc1 loads).  No block waits for another.  The words live
// in a per-device pool, a rotating slot per launch, reset by the last arriver (graph replay).
// (A variant where the last C/16 arrivers of the BN backward reduce / tensor statistics passes
// polled until every block had arrived and then folded 256 KB each measured slower: r6 below.)
typedef __attribute__((address_space(1))) unsigned gu32;
typedef __attribute__((address_space(1))) unsigned long long gu64;
constexpr int TK_SLOTS = 256, TK_WORDS = 128;        // C / 16 <= 128 groups per launch
__device__ unsigned fv_bn_tickets[TK_SLOTS * TK_WORDS];

__device__ __forceinline__ void st_sc1_f64(double* p, double v) {
  __hip_atomic_store((gu64*)p, (unsigned long long)__double_as_longlong(v), __ATOMIC_RELAXED,
                     __HIP_MEMORY_SCOPE_AGENT);
}
__device__ __forceinline__ double ld_sc1_f64(const double* p) {
  return __longlong_as_double(
      (long long)__hip_atomic_load((gu64*)const_cast<double*>(p), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT));
}

template <int NV, int MODE>
__global__ void __launch_bounds__(256) fold16_part_kernel(FoldArgs a, int rows, double* part, unsigned* tk) {
  const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
  const int c0 = blockIdx.x * 16, ch = blockIdx.y, q = lane & 3;
  const int r0 = ch * rows, r1 = min(a.nrec, r0 + rows);
  const float* src = reinterpret_cast<const float*>(a.src) + c0 + 4 * q;
  double acc[NV][4];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int k = 0; k < 4; ++k) acc[v][k] = 0.0;
#pragma unroll 4
  for (int r = r0 + (lane >> 2) + 16 * w; r < r1; r += 64) {
    const float* p = src + (long)r * a.rstride;
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      const float4 f = *reinterpret_cast<const float4*>(p + (long)v * a.C);
      acc[v][0] += f.x; acc[v][1] += f.y; acc[v][2] += f.z; acc[v][3] += f.w;
    }
  }
  // lanes with the same q hold the same 4 channels: xor over the 16 row lanes of the wave
  __shared__ double red[4][NV][16];
#pragma unroll
  for (int v = 0; v < NV; ++v)
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      double t = acc[v][k];
#pragma unroll
      for (int o = 4; o < 64; o <<= 1) t += __shfl_xor(t, o, 64);
      if (lane < 4) red[w][v][4 * lane + k] = t;
    }
  __syncthreads();
  if (w != 0) return;
  if (tid < 16) {
#pragma unroll
    for (int v = 0; v < NV; ++v) {
      double t = 0.0;
#pragma unroll
      for (int j = 0; j < 4; ++j) t += red[j][v][tid];
      st_sc1_f64(part + ((long)ch * NV + v) * a.C + c0 + tid, t);
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  unsigned t = 0;
  if (lane == 0) t = __hip_atomic_fetch_add((gu32*)(tk + blockIdx.x), 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  t = __shfl(t, 0, 64);
  if (t != gridDim.y - 1) return;
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
  // lane = (chunk lane rl, channel): chunks rl, rl + 4, ... (loads of 4 chunks in flight), then
  // the xor tree over the 4 chunk lanes
  const int cl = lane & 15, rl = lane >> 4, nch = gridDim.y;
  double tot[NV];
#pragma unroll
  for (int v = 0; v < NV; ++v) tot[v] = 0.0;
#pragma unroll 4
  for (int r = rl; r < nch; r += 4)
#pragma unroll
    for (int v = 0; v < NV; ++v) tot[v] += ld_sc1_f64(part + ((long)r * NV + v) * a.C + c0 + cl);
#pragma unroll
  for (int v = 0; v < NV; ++v) {
    tot[v] += __shfl_xor(tot[v], 16, 64);
    tot[v] += __shfl_xor(tot[v], 32, 64);
  }
  if (lane < 16) fold_finish<NV, MODE>(a, c0 + lane, tot);
  if (lane == 0) __hip_atomic_store((gu32*)(tk + blockIdx.x), 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int NV, int MODE>
__device__ __forceinline__ void fold_finish(const FoldArgs& a, int c, const double* tot) {
  // (n, S, Q): rows with a count row carry it first; fp32 records are counted by P
  const double n = NV == 3 ? tot[0] : (double)a.P;
  const double S = tot[NV - 2], Q = tot[NV - 1];
  if constexpr (MODE == FOLD_STATS) {
    a.stats[c] = n;
    a.stats[a.C + c] = S;
    a.stats[2 * a.C + c] = Q;
  } else if constexpr (MODE == FOLD_FWD) {
    if (a.nbt && c == 0) a.nbt[0] += 1;
    bn_finalize_one(c, a.C, n, S, Q, a.gamma, a.beta, a.eps, a.mom, 1, a.rm, a.rv, a.save_mean, a.save_invstd,
                    a.scale, a.shift);
  } else {
    // backward rows are (sum g, sum g * yhat)
    if (a.dbeta) a.dbeta[c] = (float)S;
    if (a.dgamma) a.dgamma[c] = (float)Q;
    if (a.k && a.count > 0) {
      a.k[c] = (float)(S / a.count);
      a.k[a.C + c] = (float)(Q / a.count);
    }
    if (a.red) {
      a.red[c] = S;
      a.red[a.C + c] = Q;
    }
  }
}

// the arrival words of one two-level fold launch: a rotating slot of the per-device pool, so
// launches in flight on different streams never share one (a captured launch keeps its slot;
// the kernel leaves it zeroed)
unsigned* ticket_slot() {
  static unsigned* base[64] = {};
  static std::atomic<unsigned> next{0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return nullptr;
  if (!base[dev] && hipGetSymbolAddress((void**)&base[dev], HIP_SYMBOL(fv_bn_tickets)) != hipSuccess) return nullptr;
  return base[dev] + (next.fetch_add(1) % TK_SLOTS) * TK_WORDS;
}

// scratch: room for max(ceil(nrec / FOLDR), ceil(256 / (C / 16)) + 1) x NV x C doubles (fp32
// records and rows beyond FOLD2 fold in two launches: chunk partials, then the partial rows)
template <typename T, int NV, int MODE>
int launch_fold(const FoldArgs& a, hipStream_t s, const char* what, double* scratch = nullptr) {
  FV_REQUIRE(a.C % 8 == 0 && a.nrec > 0, "BN fold: channels must be a multiple of 8 (%d)", a.C);
  const int nch = (a.nrec + FOLDR - 1) / FOLDR;
  if (sizeof(T) == 4 && scratch && (const void*)scratch != a.src && a.C % 16 == 0 && a.rstride % 4 == 0 &&
      a.nrec >= 256) {
    // fp32 records: two levels over 16-channel segments, enough (group, chunk) blocks to cover
    // the CUs (r4: res-conv folds 13.1 -> 5.4 + 5.1 us, step 12.55 -> 12.48 ms)
    const int ng = a.C / 16;
    int nch = (256 + ng - 1) / ng;
    if (nch > a.nrec / 64) nch = a.nrec / 64;
    const int rows = (a.nrec + nch - 1) / nch;
    nch = (a.nrec + rows - 1) / rows;
    unsigned* tk = ticket_slot();
    FV_REQUIRE(tk && ng <= TK_WORDS, "BN fold: no ticket slot");
    hipLaunchKernelGGL((fold16_part_kernel<NV, MODE>), dim3(ng, nch), dim3(256), 0, s, a, rows, scratch, tk);
    return fv_check_launch(what);
  }
  if (a.nrec <= FOLD2) {
    if (a.C % 16 == 0) hipLaunchKernelGGL((fold16_kernel<T, NV, MODE>), dim3(a.C / 16), dim3(FOLDT), 0, s, a);
    else hipLaunchKernelGGL((fold1_kernel<T, NV, MODE>), dim3(a.C), dim3(FOLDT), 0, s, a);
    return fv_check_launch(what);
  }
  FV_REQUIRE(scratch && (const void*)scratch != a.src, "BN fold of %d records: no scratch", a.nrec);
  hipLaunchKernelGGL((fold_part_kernel<T, NV>), dim3(a.C / 8, nch), dim3(FOLDB), 0, s, a, scratch);
  FoldArgs b = a;
  b.src = scratch;
  b.nrec = nch;
  b.rstride = (long)NV * a.C;
  hipLaunchKernelGGL((fold1_kernel<double, NV, MODE>), dim3(a.C), dim3(FOLDT), 0, s, b);
  return fv_check_launch(what);
}

// out = [pool](act(y*scale+shift)).  grid.y = output row (n*Ho + i), grid.x covers the row's
// (pixel, 8-channel chunk) pairs: 32-bit shift/mask indexing only.
template <typename T>
__global__ void act_fwd_kernel(const T* __restrict__ y, int W, int C, int ldc, int lgcpc,
                               const float* __restrict__ scale, const float* __restrict__ shift,
                               float slope, int pool, T* __restrict__ out) {
  const int Wo = pool ? W >> 1 : W;
  const int e = blockIdx.x * NTH + threadIdx.x;
  if (e >= (Wo << lgcpc)) return;
  const int row = blockIdx.y;
  const int j = e >> lgcpc, c = (e & ((1 << lgcpc) - 1)) * 8;
  float sc[8], sh[8];
  {
    const float4 a0 = *reinterpret_cast<const float4*>(scale + c), a1 = *reinterpret_cast<const float4*>(scale + c + 4);
    const float4 b0 = *reinterpret_cast<const float4*>(shift + c), b1 = *reinterpret_cast<const float4*>(shift + c + 4);
    sc[0] = a0.x; sc[1] = a0.y; sc[2] = a0.z; sc[3] = a0.w; sc[4] = a1.x; sc[5] = a1.y; sc[6] = a1.z; sc[7] = a1.w;
    sh[0] = b0.x; sh[1] = b0.y; sh[2] = b0.z; sh[3] = b0.w; sh[4] = b1.x; sh[5] = b1.y; sh[6] = b1.z; sh[7] = b1.w;
  }
  float o[8];
  if (!pool) {
    float f[8];
    ld8<T>(y + (size_t)(row * W + j) * ldc + c, f);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = fv_act(f[q] * sc[q] + sh[q], slope);
  } else {
    float f0[8], f1[8], f2[8], f3[8];
    const size_t r0 = (size_t)(2 * row) * W + 2 * j, r1 = r0 + W;
    ld8<T>(y + r0 * ldc + c, f0);
    ld8<T>(y + (r0 + 1) * ldc + c, f1);
    ld8<T>(y + r1 * ldc + c, f2);
    ld8<T>(y + (r1 + 1) * ldc + c, f3);
#pragma unroll
    for (int q = 0; q < 8; ++q)
      o[q] = 0.25f * ((fv_act(f0[q] * sc[q] + sh[q], slope) + fv_act(f1[q] * sc[q] + sh[q], slope)) +
                      (fv_act(f2[q] * sc[q] + sh[q], slope) + fv_act(f3[q] * sc[q] + sh[q], slope)));
  }
  st8<T>(out + (size_t)(row * Wo + j) * C + c, o);
}

// act_fwd (no pool, dense channels) that also writes an e4m3 copy of its output for an fp8 conv:
// the bf16-rounded output quantized with the delayed scale of the consumer's site (exactly what
// a separate quantize pass over `out` would write), the block amax into the site's in-flight
// slot.  Flat grid-stride over 8-channel chunks; the stride is a multiple of C/8, so each thread
// keeps one chunk's scale / shift.
template <typename T>
__global__ void __launch_bounds__(NTH) act_fwd_q8_kernel(const T* __restrict__ y, int n8, int lgcpc,
                                                         const float* __restrict__ scale,
                                                         const float* __restrict__ shift, float slope,
                                                         T* __restrict__ out, uint8_t* __restrict__ out8,
                                                         unsigned* st) {
  const float s = pow2_scale_of(site_hist_max(st));
  if (blockIdx.x == 0 && threadIdx.x == 0) st[18] = __float_as_uint(1.f / s);
  const int e0 = blockIdx.x * NTH + threadIdx.x;
  const int c = (e0 & ((1 << lgcpc) - 1)) * 8;
  float sc[8], sh[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    sc[q] = scale[c + q];
    sh[q] = shift[c + q];
  }
  float m = 0.f;
  for (int e = e0; e < n8; e += gridDim.x * NTH) {
    float f[8], o[8];
    ld8<T>(y + (size_t)e * 8, f);
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = fv_act(f[q] * sc[q] + sh[q], slope);
    Chunk8<T> ch;
    ch.set8(o);
    if (out) ch.store(out + (size_t)e * 8);             // (NULL: the e4m3 copy only)
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = ch.get(q);
    *reinterpret_cast<uint2*>(out8 + (size_t)e * 8) = q8_pack(o, s, m);
  }
  q8_block_amax(m, st);
}

// per-thread copy of one 8-channel chunk's BN parameters
struct BnChunk {
  float mean[8], inv[8], gam[8], bet[8];
  __device__ __forceinline__ void load(const float* m, const float* iv, const float* g, const float* b, int c) {
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      mean[q] = m[c + q];
      inv[q] = iv[c + q];
      gam[q] = g[c + q];
      bet[q] = b[c + q];
    }
  }
};

// g = dout_full * act'(gamma*yhat + beta) at pixel p (pooled dout: [P/4][C], 0.25 per tap)
template <typename T>
__device__ __forceinline__ void grad_g(const T* dout, const T* y, int p, FastDiv fw, int W, int C, int ldc,
                                       int c, int pool, const BnChunk& bp, float slope, float* g, float* yh) {
  float d[8], v[8];
  if (pool) {
    const int hr = (int)fdiv((uint32_t)p, fw);            // n*H + h
    const int w = p - hr * W;
    ld8<T>(dout + (size_t)((hr >> 1) * (W >> 1) + (w >> 1)) * C + c, d);
#pragma unroll
    for (int q = 0; q < 8; ++q) d[q] *= 0.25f;
  } else {
    ld8<T>(dout + (size_t)p * ldc + c, d);
  }
  ld8<T>(y + (size_t)p * ldc + c, v);
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    yh[q] = (v[q] - bp.mean[q]) * bp.inv[q];
    const float z = bp.gam[q] * yh[q] + bp.bet[q];
    g[q] = z > 0.f ? d[q] : d[q] * slope;
  }
}

template <typename T>
__global__ void act_bwd_reduce_kernel(const T* __restrict__ dout, const T* __restrict__ y, int P, FastDiv fw,
                                      int W, int C, int ldc, const float* mean, const float* invstd,
                                      const float* gamma, const float* beta, float slope, int pool,
                                      double* ws) {
  const int tpp = C / 8;
  const int rows = NTH / tpp;
  const int cg = threadIdx.x % tpp, row = threadIdx.x / tpp;
  BnChunk bp;
  bp.load(mean, invstd, gamma, beta, cg * 8);
  float s[8], q2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q2[j] = 0.f;
  // two pixels per iteration: four independent 16-B loads in flight per thread (one pair was
  // latency bound on the 256x256 layers: 3.9-4.3 TB/s against 5.3-5.7 for the apply pass)
  const int stride = gridDim.x * rows;
  int p = blockIdx.x * rows + row;
  for (; p + stride < P; p += 2 * stride) {
    float g[8], yh[8], g2[8], yh2[8];
    grad_g<T>(dout, y, p, fw, W, C, ldc, cg * 8, pool, bp, slope, g, yh);
    grad_g<T>(dout, y, p + stride, fw, W, C, ldc, cg * 8, pool, bp, slope, g2, yh2);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += g[j] + g2[j];
      q2[j] += g[j] * yh[j] + g2[j] * yh2[j];
    }
  }
  if (p < P) {
    float g[8], yh[8];
    grad_g<T>(dout, y, p, fw, W, C, ldc, cg * 8, pool, bp, slope, g, yh);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += g[j];
      q2[j] += g[j] * yh[j];
    }
  }
  __shared__ float ss[2][NTH * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss[0][row * C + cg * 8 + j] = s[j];
    ss[1][row * C + cg * 8 + j] = q2[j];
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

// Pooled layers (DownBlock2D: conv -> BN -> act -> AvgPool2d(2)): one thread per (2x2 quad,
// 8-channel chunk), so the pooled output gradient is loaded once for its four pixels (the
// per-pixel kernels above load it four times and divide every pixel index by W): 5 loads in
// flight per iteration, not 8.  Quad q = (n*Ho + ho)*Wo + wo covers pixels (2ho + i, 2wo + j).
template <typename T>
__device__ __forceinline__ void quad_g(const T* dout, const T* y, int q, FastDiv fwo, int W, int C, int c,
                                       const BnChunk& bp, float slope, float (&g)[4][8], float (&yh)[4][8],
                                       int (&pix)[4]) {
  const int hr = (int)fdiv((uint32_t)q, fwo);           // n*Ho + ho
  const int wo = q - hr * (W >> 1);
  pix[0] = (2 * hr) * W + 2 * wo;
  pix[1] = pix[0] + 1;
  pix[2] = pix[0] + W;
  pix[3] = pix[2] + 1;
  float d[8], v[4][8];
  ld8<T>(dout + (size_t)q * C + c, d);
#pragma unroll
  for (int t = 0; t < 4; ++t) ld8<T>(y + (size_t)pix[t] * C + c, v[t]);
#pragma unroll
  for (int t = 0; t < 4; ++t)
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      yh[t][u] = (v[t][u] - bp.mean[u]) * bp.inv[u];
      const float z = bp.gam[u] * yh[t][u] + bp.bet[u];
      const float dq = 0.25f * d[u];
      g[t][u] = z > 0.f ? dq : dq * slope;
    }
}

template <typename T>
__global__ void act_bwd_reduce_pool_kernel(const T* __restrict__ dout, const T* __restrict__ y, int Pq, FastDiv fwo,
                                           int W, int C, const float* mean, const float* invstd,
                                           const float* gamma, const float* beta, float slope, double* ws) {
  const int tpp = C / 8;
  const int rows = NTH / tpp;
  const int cg = threadIdx.x % tpp, row = threadIdx.x / tpp;
  BnChunk bp;
  bp.load(mean, invstd, gamma, beta, cg * 8);
  float s[8], q2[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) s[j] = q2[j] = 0.f;
  for (int q = blockIdx.x * rows + row; q < Pq; q += gridDim.x * rows) {
    float g[4][8], yh[4][8];
    int pix[4];
    quad_g<T>(dout, y, q, fwo, W, C, cg * 8, bp, slope, g, yh, pix);
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      s[j] += (g[0][j] + g[1][j]) + (g[2][j] + g[3][j]);
      q2[j] += (g[0][j] * yh[0][j] + g[1][j] * yh[1][j]) + (g[2][j] * yh[2][j] + g[3][j] * yh[3][j]);
    }
  }
  __shared__ float ss[2][NTH * 8];
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    ss[0][row * C + cg * 8 + j] = s[j];
    ss[1][row * C + cg * 8 + j] = q2[j];
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

template <typename T>
__global__ void act_bwd_apply_pool_kernel(const T* __restrict__ dout, const T* __restrict__ y, int Pq, FastDiv fwo,
                                          int W, int C, int lgcpc, const float* mean, const float* invstd,
                                          const float* gamma, const float* beta, float slope,
                                          const float* __restrict__ k, const T* __restrict__ addend,
                                          T* __restrict__ dx) {
  const int total = Pq << lgcpc;
  const int e0 = blockIdx.x * NTH + threadIdx.x;
  const int c = (e0 & ((1 << lgcpc) - 1)) * 8;
  BnChunk bp;
  bp.load(mean, invstd, gamma, beta, c);
  float k0[8], k1[8], gi[8];
#pragma unroll
  for (int u = 0; u < 8; ++u) {
    k0[u] = k[c + u];
    k1[u] = k[C + c + u];
    gi[u] = bp.gam[u] * bp.inv[u];
  }
  for (int e = e0; e < total; e += gridDim.x * NTH) {
    const int q = e >> lgcpc;
    float g[4][8], yh[4][8];
    int pix[4];
    quad_g<T>(dout, y, q, fwo, W, C, c, bp, slope, g, yh, pix);
#pragma unroll
    for (int t = 0; t < 4; ++t) {
      float o[8], ad[8];
      if (addend) ld8<T>(addend + (size_t)pix[t] * C + c, ad);
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        o[u] = gi[u] * (g[t][u] - k0[u] - yh[t][u] * k1[u]);
        if (addend) o[u] += ad[u];
      }
      st8<T>(dx + (size_t)pix[t] * C + c, o);
    }
  }
}

// cnt (optional): per-channel element count on the device (row 0 of the all-reduced [3][C]
// statistics record: the global count even with uneven per-rank batches); k may be NULL
// (dgamma / dbeta only)
__global__ void bwd_finalize_kernel(const double* red, int C, double count, const double* cnt, float* dgamma,
                                    float* dbeta, float* k) {
  const int c = blockIdx.x * blockDim.x + threadIdx.x;
  if (c >= C) return;
  const double sg = red[c], sgy = red[C + c];
  if (dbeta) dbeta[c] = (float)sg;
  if (dgamma) dgamma[c] = (float)sgy;
  if (k) {
    const double n = cnt ? cnt[c] : count;
    k[c] = (float)(sg / n);
    k[C + c] = (float)(sgy / n);
  }
}

// dx = gamma*invstd*(g - k0 - yhat*k1) [+ addend]; thread = (pixel, 8-channel chunk), the
// grid stride is a multiple of C/8 so each thread keeps one chunk's parameters in registers
template <typename T>
__global__ void act_bwd_apply_kernel(const T* __restrict__ dout, const T* __restrict__ y, int P, FastDiv fw,
                                     int W, int C, int ldc, int lgcpc, const float* mean, const float* invstd,
                                     const float* gamma, const float* beta, float slope, int pool,
                                     const float* __restrict__ k, const T* __restrict__ addend, T* __restrict__ dx) {
  const int total = P << lgcpc;
  const int e0 = blockIdx.x * NTH + threadIdx.x;
  const int c = (e0 & ((1 << lgcpc) - 1)) * 8;
  BnChunk bp;
  bp.load(mean, invstd, gamma, beta, c);
  float k0[8], k1[8], gi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    k0[q] = k[c + q];
    k1[q] = k[C + c + q];
    gi[q] = bp.gam[q] * bp.inv[q];
  }
  for (int e = e0; e < total; e += gridDim.x * NTH) {
    const int p = e >> lgcpc;
    float g[8], yh[8], o[8];
    grad_g<T>(dout, y, p, fw, W, C, ldc, c, pool, bp, slope, g, yh);
    float ad[8];
    if (addend) ld8<T>(addend + (size_t)p * ldc + c, ad);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[q] = gi[q] * (g[q] - k0[q] - yh[q] * k1[q]);
      if (addend) o[q] += ad[q];
    }
    st8<T>(dx + (size_t)p * ldc + c, o);
  }
}

// act_bwd_apply (no pool, dense channels) that also writes the e4m3 copy of dx for the fp8 data
// gradient consuming it (see act_fwd_q8_kernel)
template <typename T>
__global__ void __launch_bounds__(NTH) act_bwd_apply_q8_kernel(
    const T* __restrict__ dout, const T* __restrict__ y, int P, int C, int lgcpc, const float* mean,
    const float* invstd, const float* gamma, const float* beta, float slope, const float* __restrict__ k,
    const T* __restrict__ addend, T* __restrict__ dx, uint8_t* __restrict__ dx8, unsigned* st) {
  const float s = pow2_scale_of(site_hist_max(st));
  if (blockIdx.x == 0 && threadIdx.x == 0) st[18] = __float_as_uint(1.f / s);
  const int total = P << lgcpc;
  const int e0 = blockIdx.x * NTH + threadIdx.x;
  const int c = (e0 & ((1 << lgcpc) - 1)) * 8;
  BnChunk bp;
  bp.load(mean, invstd, gamma, beta, c);
  float k0[8], k1[8], gi[8];
#pragma unroll
  for (int q = 0; q < 8; ++q) {
    k0[q] = k[c + q];
    k1[q] = k[C + c + q];
    gi[q] = bp.gam[q] * bp.inv[q];
  }
  const FastDiv unused = {0u, 0u};
  float m = 0.f;
  for (int e = e0; e < total; e += gridDim.x * NTH) {
    const int p = e >> lgcpc;
    float g[8], yh[8], o[8];
    grad_g<T>(dout, y, p, unused, 0, C, C, c, 0, bp, slope, g, yh);
    float ad[8];
    if (addend) ld8<T>(addend + (size_t)p * C + c, ad);
#pragma unroll
    for (int q = 0; q < 8; ++q) {
      o[q] = gi[q] * (g[q] - k0[q] - yh[q] * k1[q]);
      if (addend) o[q] += ad[q];
    }
    Chunk8<T> ch;
    ch.set8(o);
    if (dx) ch.store(dx + (size_t)p * C + c);           // (NULL: the e4m3 copy only)
#pragma unroll
    for (int q = 0; q < 8; ++q) o[q] = ch.get(q);
    *reinterpret_cast<uint2*>(dx8 + (size_t)p * C + c) = q8_pack(o, s, m);
  }
  q8_block_amax(m, st);
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
  FV_REQUIRE((long)nblocks * block_pixels >= total_pixels, "bn_stats_from_partials: records do not cover the pixels");
  FoldArgs a{};
  a.src = partials; a.nrec = nblocks; a.C = c; a.rstride = 2L * c; a.P = total_pixels; a.stats = stats;
  return launch_fold<float, 2, FOLD_STATS>(a, (hipStream_t)stream, "bn_fold_stats", (double*)ws);
}

int fv_bn_bwd_from_records(const float* records, int nrec, int record_pixels, long pixels, int c, long count,
                           float* dgamma, float* dbeta, float* k, double* red, void* ws, void* stream) {
  FV_REQUIRE(records && ws && nrec > 0 && c > 0 && (long)nrec * record_pixels == pixels,
             "bn_bwd_from_records: bad arguments");
  FoldArgs a{};
  a.src = records; a.nrec = nrec; a.C = c; a.rstride = 2L * c;
  a.count = (double)count; a.dgamma = dgamma; a.dbeta = dbeta; a.k = k; a.red = red;
  return launch_fold<float, 2, FOLD_BWD>(a, (hipStream_t)stream, "bn_bwd_fold_records", (double*)ws);
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
  FoldArgs a{};
  a.src = ws; a.nrec = nb; a.C = c; a.rstride = 3L * c; a.stats = stats;
  return launch_fold<double, 3, FOLD_STATS>(a, s, "bn_fold_tensor_stats");
}

int fv_bn_finalize(const double* stats, int c, const float* gamma, const float* beta, float eps,
                   float momentum, int training, float* running_mean, float* running_var,
                   long long* num_batches_tracked, float* save_mean, float* save_invstd, float* scale,
                   float* shift, void* stream) {
  FV_REQUIRE(c > 0, "bad channels");
  FV_REQUIRE(!training || stats, "training finalize needs stats");
  FV_REQUIRE(training || (running_mean && running_var), "eval finalize needs running stats");
  hipLaunchKernelGGL(finalize_kernel, dim3(fv_cdiv(c, NTH)), dim3(NTH), 0, (hipStream_t)stream, stats, c, gamma,
                     beta, eps, momentum, training, running_mean, running_var, num_batches_tracked, save_mean,
                     save_invstd, scale, shift);
  return fv_check_launch("bn_finalize");
}

int fv_bn_stats_finalize_partials(const float* partials, int nblocks, int block_pixels, long total_pixels, int c,
                                  const float* gamma, const float* beta, float eps, float momentum,
                                  float* running_mean, float* running_var, long long* num_batches_tracked,
                                  float* save_mean, float* save_invstd, float* scale, float* shift, void* ws,
                                  void* stream) {
  FV_REQUIRE(partials, "null pointer");
  FV_REQUIRE(nblocks > 0 && c > 0, "bad sizes");
  FV_REQUIRE((long)nblocks * block_pixels >= total_pixels, "bn_stats_finalize_partials: records do not cover the pixels");
  FoldArgs a{};
  a.src = partials; a.nrec = nblocks; a.C = c; a.rstride = 2L * c; a.P = total_pixels;
  a.gamma = gamma; a.beta = beta; a.eps = eps; a.mom = momentum; a.rm = running_mean; a.rv = running_var;
  a.nbt = num_batches_tracked; a.save_mean = save_mean; a.save_invstd = save_invstd; a.scale = scale; a.shift = shift;
  return launch_fold<float, 2, FOLD_FWD>(a, (hipStream_t)stream, "bn_fold_finalize", (double*)ws);
}

int fv_bn_stats_finalize_tensor(int dtype, const void* x, long pixels, int c, int ldc, const float* gamma,
                                const float* beta, float eps, float momentum, float* running_mean,
                                float* running_var, long long* num_batches_tracked, float* save_mean,
                                float* save_invstd, float* scale, float* shift, void* ws, void* stream) {
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(x && ws, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const int nb = stream_blocks(pixels, c);
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(tensor_stats_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)x, pixels, c, ldc,
                       (double*)ws);
  else
    hipLaunchKernelGGL(tensor_stats_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)x, pixels, c, ldc,
                       (double*)ws);
  if ((st = fv_check_launch("bn_tensor_stats"))) return st;
  FoldArgs a{};
  a.src = ws; a.nrec = nb; a.C = c; a.rstride = 3L * c;
  a.gamma = gamma; a.beta = beta; a.eps = eps; a.mom = momentum; a.rm = running_mean; a.rv = running_var;
  a.nbt = num_batches_tracked; a.save_mean = save_mean; a.save_invstd = save_invstd; a.scale = scale; a.shift = shift;
  return launch_fold<double, 3, FOLD_FWD>(a, s, "bn_fold_tensor_finalize");
}

int fv_bn_act_fwd(int dtype, const void* y, int n, int h, int w, int c, int ldc, const float* scale,
                  const float* shift, float slope, int pool, void* out, void* stream) {
  FV_REQUIRE(fv_slope_ok(slope), "activation slope must be in [0, 1] (got %g)", (double)slope);
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(!pool || (h % 2 == 0 && w % 2 == 0), "pool needs even h, w");
  FV_REQUIRE((long)n * h * w * ldc < (1L << 31), "bn: tensor too large for 32-bit indexing");
  const int lgcpc = fv_ilog2(c / 8);
  const int ho = pool ? h / 2 : h, wo = pool ? w / 2 : w;
  FV_REQUIRE(n * ho <= 65535, "bn: too many rows");
  const dim3 grid(fv_cdiv((long)wo << lgcpc, NTH), n * ho);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(act_fwd_kernel<bf16>, grid, dim3(NTH), 0, s, (const bf16*)y, w, c, ldc, lgcpc, scale, shift,
                       slope, pool, (bf16*)out);
  else
    hipLaunchKernelGGL(act_fwd_kernel<float>, grid, dim3(NTH), 0, s, (const float*)y, w, c, ldc, lgcpc, scale,
                       shift, slope, pool, (float*)out);
  return fv_check_launch("bn_act_fwd");
}

int fv_bn_act_bwd_reduce(int dtype, const void* dout, const void* y, int n, int h, int w, int c, int ldc,
                         const float* mean, const float* invstd, const float* gamma, const float* beta,
                         float slope, int pool, double* red, void* ws, void* stream) {
  FV_REQUIRE(fv_slope_ok(slope), "activation slope must be in [0, 1] (got %g)", (double)slope);
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(!pool || ldc == c, "pooled bwd needs dense channels");
  hipStream_t s = (hipStream_t)stream;
  FV_REQUIRE((long)n * h * w * ldc < (1L << 31), "bn: tensor too large for 32-bit indexing");
  const int nb = stream_blocks((long)n * h * w, c);
  const int P = n * h * w;
  const FastDiv fw = make_fastdiv((uint32_t)w);
  if (pool) {   // 2x2-quad kernels (even H, W: AvgPool2d(2) requires them)
    FV_REQUIRE(h % 2 == 0 && w % 2 == 0, "pooled bwd needs even h, w");
    const int Pq = P / 4;
    const FastDiv fwo = make_fastdiv((uint32_t)(w / 2));
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(act_bwd_reduce_pool_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)dout,
                         (const bf16*)y, Pq, fwo, w, c, mean, invstd, gamma, beta, slope, (double*)ws);
    else
      hipLaunchKernelGGL(act_bwd_reduce_pool_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)dout,
                         (const float*)y, Pq, fwo, w, c, mean, invstd, gamma, beta, slope, (double*)ws);
  } else {
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(act_bwd_reduce_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)dout,
                         (const bf16*)y, P, fw, w, c, ldc, mean, invstd, gamma, beta, slope, pool, (double*)ws);
    else
      hipLaunchKernelGGL(act_bwd_reduce_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)dout,
                         (const float*)y, P, fw, w, c, ldc, mean, invstd, gamma, beta, slope, pool, (double*)ws);
  }
  if ((st = fv_check_launch("bn_bwd_reduce"))) return st;
  FoldArgs a{};
  a.src = ws; a.nrec = nb; a.C = c; a.rstride = 2L * c; a.red = red;
  return launch_fold<double, 2, FOLD_BWD>(a, s, "bn_bwd_fold");
}

int fv_bn_act_bwd_reduce_finalize(int dtype, const void* dout, const void* y, int n, int h, int w, int c,
                                  int ldc, const float* mean, const float* invstd, const float* gamma,
                                  const float* beta, float slope, int pool, long count, float* dgamma,
                                  float* dbeta, float* k, void* ws, void* stream) {
  FV_REQUIRE(fv_slope_ok(slope), "activation slope must be in [0, 1] (got %g)", (double)slope);
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(!pool || ldc == c, "pooled bwd needs dense channels");
  FV_REQUIRE(k && ws && count > 0, "bad args");
  hipStream_t s = (hipStream_t)stream;
  FV_REQUIRE((long)n * h * w * ldc < (1L << 31), "bn: tensor too large for 32-bit indexing");
  const int nb = stream_blocks((long)n * h * w, c);
  const int P = n * h * w;
  const FastDiv fw = make_fastdiv((uint32_t)w);
  if (pool) {   // 2x2-quad kernels (even H, W: AvgPool2d(2) requires them)
    FV_REQUIRE(h % 2 == 0 && w % 2 == 0, "pooled bwd needs even h, w");
    const int Pq = P / 4;
    const FastDiv fwo = make_fastdiv((uint32_t)(w / 2));
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(act_bwd_reduce_pool_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)dout,
                         (const bf16*)y, Pq, fwo, w, c, mean, invstd, gamma, beta, slope, (double*)ws);
    else
      hipLaunchKernelGGL(act_bwd_reduce_pool_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)dout,
                         (const float*)y, Pq, fwo, w, c, mean, invstd, gamma, beta, slope, (double*)ws);
  } else {
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(act_bwd_reduce_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)dout,
                         (const bf16*)y, P, fw, w, c, ldc, mean, invstd, gamma, beta, slope, pool, (double*)ws);
    else
      hipLaunchKernelGGL(act_bwd_reduce_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)dout,
                         (const float*)y, P, fw, w, c, ldc, mean, invstd, gamma, beta, slope, pool, (double*)ws);
  }
  if ((st = fv_check_launch("bn_bwd_reduce"))) return st;
  FoldArgs a{};
  a.src = ws; a.nrec = nb; a.C = c; a.rstride = 2L * c;
  a.count = (double)count; a.dgamma = dgamma; a.dbeta = dbeta; a.k = k;
  return launch_fold<double, 2, FOLD_BWD>(a, s, "bn_bwd_fold_finalize");
}

int fv_bn_bwd_finalize(const double* red, int c, long count, float* dgamma, float* dbeta, float* k,
                       void* stream) {
  FV_REQUIRE(red && (k || dgamma || dbeta) && (!k || count > 0), "bad args");
  hipLaunchKernelGGL(bwd_finalize_kernel, dim3(fv_cdiv(c, NTH)), dim3(NTH), 0, (hipStream_t)stream, red, c,
                     (double)count, nullptr, dgamma, dbeta, k);
  return fv_check_launch("bn_bwd_finalize");
}

int fv_bn_bwd_finalize_dev(const double* red, int c, const double* count, float* dgamma, float* dbeta, float* k,
                           void* stream) {
  FV_REQUIRE(red && count && (k || dgamma || dbeta), "bad args");
  hipLaunchKernelGGL(bwd_finalize_kernel, dim3(fv_cdiv(c, NTH)), dim3(NTH), 0, (hipStream_t)stream, red, c, 0.0,
                     count, dgamma, dbeta, k);
  return fv_check_launch("bn_bwd_finalize_dev");
}

int fv_bn_act_bwd_apply(int dtype, const void* dout, const void* y, int n, int h, int w, int c, int ldc,
                        const float* mean, const float* invstd, const float* gamma, const float* beta,
                        float slope, int pool, const float* k, const void* addend, void* dx, void* stream) {
  FV_REQUIRE(fv_slope_ok(slope), "activation slope must be in [0, 1] (got %g)", (double)slope);
  int st = check_c(c, ldc);
  if (st) return st;
  FV_REQUIRE(!pool || ldc == c, "pooled bwd needs dense channels");
  FV_REQUIRE((long)n * h * w * ldc < (1L << 31), "bn: tensor too large for 32-bit indexing");
  const long work = (long)n * h * w * (c / 8);
  const int P = n * h * w, lgcpc = fv_ilog2(c / 8);
  const FastDiv fw = make_fastdiv((uint32_t)w);
  hipStream_t s = (hipStream_t)stream;
  if (pool) {   // 2x2-quad kernels (even H, W: AvgPool2d(2) requires them)
    FV_REQUIRE(h % 2 == 0 && w % 2 == 0, "pooled bwd needs even h, w");
    const int Pq = P / 4;
    const FastDiv fwo = make_fastdiv((uint32_t)(w / 2));
    const long qwork = (long)Pq * (c / 8);
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(act_bwd_apply_pool_kernel<bf16>, dim3(grid_for(qwork, 16384)), dim3(NTH), 0, s,
                         (const bf16*)dout, (const bf16*)y, Pq, fwo, w, c, lgcpc, mean, invstd, gamma, beta, slope, k,
                         (const bf16*)addend, (bf16*)dx);
    else
      hipLaunchKernelGGL(act_bwd_apply_pool_kernel<float>, dim3(grid_for(qwork, 16384)), dim3(NTH), 0, s,
                         (const float*)dout, (const float*)y, Pq, fwo, w, c, lgcpc, mean, invstd, gamma, beta, slope,
                         k, (const float*)addend, (float*)dx);
    return fv_check_launch("bn_bwd_apply_pool");
  }
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(act_bwd_apply_kernel<bf16>, dim3(grid_for(work, 16384)), dim3(NTH), 0, s, (const bf16*)dout,
                       (const bf16*)y, P, fw, w, c, ldc, lgcpc, mean, invstd, gamma, beta, slope, pool, k,
                       (const bf16*)addend, (bf16*)dx);
  else
    hipLaunchKernelGGL(act_bwd_apply_kernel<float>, dim3(grid_for(work, 16384)), dim3(NTH), 0, s, (const float*)dout,
                       (const float*)y, P, fw, w, c, ldc, lgcpc, mean, invstd, gamma, beta, slope, pool, k,
                       (const float*)addend, (float*)dx);
  return fv_check_launch("bn_bwd_apply");
}

// fp8 (e4m3) copy of the output beside it, for a consumer conv in fp8 mode (delayed scaling:
// include/facevae.h, fv_quantize_fp8_site).  2048 blocks: one site atomic per block.
constexpr int Q8_BLOCKS = 2048;

int fv_bn_act_fwd_q8(int dtype, const void* y, int n, int h, int w, int c, const float* scale,
                     const float* shift, float slope, void* out, void* out8, void* site, void* stream) {
  FV_REQUIRE(fv_slope_ok(slope), "activation slope must be in [0, 1] (got %g)", (double)slope);
  int st = check_c(c, c);
  if (st) return st;
  FV_REQUIRE(y && scale && shift && out8 && site, "bn_act_fwd_q8: null pointer");
  const long n8 = (long)n * h * w * (c / 8);
  FV_REQUIRE(n8 * 8 < (1L << 31), "bn: tensor too large for 32-bit indexing");
  const int lgcpc = fv_ilog2(c / 8);
  const int nb = grid_for(n8, Q8_BLOCKS);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(act_fwd_q8_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)y, (int)n8, lgcpc, scale,
                       shift, slope, (bf16*)out, (uint8_t*)out8, (unsigned*)site);
  else
    hipLaunchKernelGGL(act_fwd_q8_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)y, (int)n8, lgcpc, scale,
                       shift, slope, (float*)out, (uint8_t*)out8, (unsigned*)site);
  return fv_check_launch("bn_act_fwd_q8");
}

int fv_bn_act_bwd_apply_q8(int dtype, const void* dout, const void* y, int n, int h, int w, int c,
                           const float* mean, const float* invstd, const float* gamma, const float* beta,
                           float slope, const float* k, const void* addend, void* dx, void* dx8, void* site,
                           void* stream) {
  FV_REQUIRE(fv_slope_ok(slope), "activation slope must be in [0, 1] (got %g)", (double)slope);
  int st = check_c(c, c);
  if (st) return st;
  FV_REQUIRE(dout && y && mean && invstd && gamma && beta && k && dx8 && site,
             "bn_act_bwd_apply_q8: null pointer");
  FV_REQUIRE((long)n * h * w * c < (1L << 31), "bn: tensor too large for 32-bit indexing");
  const long work = (long)n * h * w * (c / 8);
  const int P = n * h * w, lgcpc = fv_ilog2(c / 8);
  const int nb = grid_for(work, Q8_BLOCKS);
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(act_bwd_apply_q8_kernel<bf16>, dim3(nb), dim3(NTH), 0, s, (const bf16*)dout, (const bf16*)y,
                       P, c, lgcpc, mean, invstd, gamma, beta, slope, k, (const bf16*)addend, (bf16*)dx,
                       (uint8_t*)dx8, (unsigned*)site);
  else
    hipLaunchKernelGGL(act_bwd_apply_q8_kernel<float>, dim3(nb), dim3(NTH), 0, s, (const float*)dout,
                       (const float*)y, P, c, lgcpc, mean, invstd, gamma, beta, slope, k, (const float*)addend,
                       (float*)dx, (uint8_t*)dx8, (unsigned*)site);
  return fv_check_launch("bn_bwd_apply_q8");
}

}  // extern "C"
