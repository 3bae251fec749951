// Implicit-GEMM convolution for gfx950 (CDNA4): forward (+ backward-data via transposed
// weights) and backward-weight.  NHWC activations, MFMA 16x16x32 bf16 (fast mode) or
// 16x16x4 f32 (exact fp32 parity mode), fp32 accumulation.
//
// Reference behaviour replaced: F.conv2d as called by _ConvBlock / nn.Conv2d
// (modules.py:32-42; models.py:932-934, 1095-1099) in the FaceVAE path, plus the fused
// pieces around it (nearest x2 upsample modules.py:81, NAC BN-apply+act modules.py:13,
// residual add modules.py:125, sigmoid models.py:1110, BN statistics modules.py:19).
//
// Forward GEMM orientation:  D[co][pixel] = W[co][k] * im2col(x)[k][pixel]
//   MFMA A operand = weight tile (rows = output channels), B operand = activation tile
//   (cols = pixels).  The accumulator layout then gives each lane 4 consecutive output
//   channels of one pixel -> contiguous NHWC stores.  K = (tap, ci), ci fastest, chunks
//   of 8 k never straddle a tap (cin is a power of two >= 8).
#include <stdlib.h>

#include <algorithm>
#include <type_traits>

#include "common.h"

namespace {

constexpr int BK = 32;  // k per main-loop step (one bf16 MFMA K, eight f32 MFMA K=4)

// Diagnostic build only (build.py --diag -> libfacevae_diag.so, tools/convbench.py --diag):
// per-wave shader-clock stamps of the res conv kernel into a device table read back with
// fv_diag_read.  The production library compiles none of this.
#ifdef FV_DIAG
constexpr int DIAG_SLOTS = 8;
__device__ unsigned long long g_diag[4096 * 8 * DIAG_SLOTS];
#define FV_DIAG_T(var) const unsigned long long var = __builtin_amdgcn_s_memtime()
#define FV_DIAG_PUT(slot, val)                                                                     \
  do {                                                                                             \
    const unsigned long long v_ = (val);                                                           \
    if ((threadIdx.x & 63) == 0 && blockIdx.x < 4096)                                              \
      g_diag[((size_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) * DIAG_SLOTS + (slot)] = v_; \
  } while (0)
// kernel entry / after the prologue barrier / around each main-loop wait + barrier / after
// the post-barrier issue block / after the main loop / at the end
#define FV_DIAG_BEGIN()                                                \
  FV_DIAG_T(d_t0);                                                     \
  const unsigned long long d_r0 = __builtin_amdgcn_s_memrealtime();    \
  unsigned long long d_tw = 0, d_ti = 0, d_wb = 0
#define FV_DIAG_PROLOGUE() FV_DIAG_T(d_t1)
#define FV_DIAG_WAIT_BEGIN() FV_DIAG_T(d_wa)
#define FV_DIAG_WAIT_END()                   \
  do {                                       \
    d_wb = __builtin_amdgcn_s_memtime();     \
    d_tw += d_wb - d_wa;                     \
  } while (0)
#define FV_DIAG_ISSUE_END() (d_ti += __builtin_amdgcn_s_memtime() - d_wb)
#define FV_DIAG_LOOP_END() FV_DIAG_T(d_t2)
#define FV_DIAG_END()                                                                       \
  do {                                                                                      \
    FV_DIAG_T(d_t3);                                                                        \
    unsigned xcc_;                                                                          \
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(xcc_));                     \
    FV_DIAG_PUT(0, d_t0);                                                                   \
    FV_DIAG_PUT(1, d_t1);                                                                   \
    FV_DIAG_PUT(2, d_t2);                                                                   \
    FV_DIAG_PUT(3, d_t3);                                                                   \
    FV_DIAG_PUT(4, d_tw);                                                                   \
    FV_DIAG_PUT(5, d_ti);                                                                   \
    FV_DIAG_PUT(6, d_r0);                                                                   \
    FV_DIAG_PUT(7, ((unsigned long long)xcc_ << 32) | (unsigned)__builtin_amdgcn_s_memrealtime()); \
  } while (0)
#else
#define FV_DIAG_BEGIN()
#define FV_DIAG_PROLOGUE()
#define FV_DIAG_WAIT_BEGIN()
#define FV_DIAG_WAIT_END()
#define FV_DIAG_ISSUE_END()
#define FV_DIAG_LOOP_END()
#define FV_DIAG_END()
#endif

struct ConvArgs {
  const void* x;
  const void* w;
  const float* bias;
  const float* psc;
  const float* psh;
  float slope;
  const void* res;
  void* y;
  float* stats;
  int N, H, W, Hin, Win, P;
  int lgCin, Cin;
  int Cout, ldy;
  int K, Kpad, nks;
  int sigmoid, nchw;
  int ntn;
  int lgtw;       // > 0: a block's pixels are a (BM >> lgtw) x (1 << lgtw) rectangle at p0
  // sub-pixel phase of an upsample-conv (v2 MODE 2): the tile space is the LOW-res image
  // (H x W = Hin x Win, powers of two: lgw, lghw) and tile pixel (n, h, w) of phase
  // (pa, pb) stores to output pixel (n, 2h + pa, 2w + pb) of the Ho x Wo image
  int sub;        // 0 = none, else 1 + 2 * pa + pb (set per block)
  int lgw, lghw, Ho, Wo;
  int wphase;     // elements per phase block of the weight buffer (MODE 2)
  const float* dq0;   // fp8 path: per-tensor dequant factors of the two operands (device)
  const float* dq1;
  // store-pass records (STAGED epilogue, fv_store_reduce): per (m-tile, wave) and output
  // channel, 1 = (sum, sum of squares) of the stored (bf16, residual-added) output -- the next
  // BN's statistics; 2 = BN-backward sums (g, g * yhat) of the stored gradient v with
  // g = v * act'(gamma * yhat + beta), yhat = (res - mean) * invstd (`res` = the BN input,
  // prefetched like a residual, not added)
  int spm;
  float* sprec;
  const float *bnm, *bni, *bng, *bnb;
  float bns;
  int wus;        // halo 3x3 kernels: bytes per tap unit of the stage-major weights (rows * 64)
  unsigned* roll; // fp8: the operand's delayed-scaling site, rolled by block 0 (fp8_site_roll)
  int nrec;       // BN records the caller sized `stats` for (fv_conv2d_stats_blocks / fp8): every
                  // record write is bounded by it (not only by the kernel's own tiling)
};

// output pixel of tile-space pixel p (identity unless a sub-pixel phase is set)
__device__ __forceinline__ int out_pix(const ConvArgs& a, int p) {
  if (!a.sub) return p;
  const int ph = a.sub - 1, pa = ph >> 1, pb = ph & 1;
  const int n = p >> a.lghw, rem = p & ((1 << a.lghw) - 1);
  const int h = rem >> a.lgw, w = rem & ((1 << a.lgw) - 1);
  return (n * a.Ho + 2 * h + pa) * a.Wo + 2 * w + pb;
}

// 16-B chunk swizzle of a 64-B bf16 LDS row (4 chunks): conflict-free ds_read_b128 for the
// MFMA fragment read (16 consecutive rows, chunk = lane>>4).  f(row) = [0,2,3,1][(row>>2)&3].
template <typename T>
__device__ __forceinline__ int rswz(int row) {
  if constexpr (sizeof(T) == 2) return (0x1320 >> (((row >> 2) & 3) * 4)) & 3;
  else return 0;
}

template <typename T>
__device__ __forceinline__ void load4(const T* p, float* f);
template <>
__device__ __forceinline__ void load4<float>(const float* p, float* f) {
  float4 v = *reinterpret_cast<const float4*>(p);
  f[0] = v.x; f[1] = v.y; f[2] = v.z; f[3] = v.w;
}
template <>
__device__ __forceinline__ void load4<bf16>(const bf16* p, float* f) {
  uint2 v = *reinterpret_cast<const uint2*>(p);
  f[0] = __uint_as_float(v.x << 16); f[1] = __uint_as_float(v.x & 0xffff0000u);
  f[2] = __uint_as_float(v.y << 16); f[3] = __uint_as_float(v.y & 0xffff0000u);
}
template <typename T>
__device__ __forceinline__ void store4(T* p, const float* f);
template <>
__device__ __forceinline__ void store4<float>(float* p, const float* f) {
  *reinterpret_cast<float4*>(p) = make_float4(f[0], f[1], f[2], f[3]);
}
template <>
__device__ __forceinline__ void store4<bf16>(bf16* p, const float* f) {
  bf16 t[4] = {(bf16)f[0], (bf16)f[1], (bf16)f[2], (bf16)f[3]};
  *reinterpret_cast<uint2*>(p) = *reinterpret_cast<const uint2*>(t);
}

// one MFMA step over a 32-deep k slice for a 16x16 tile
template <typename T>
struct Frag;
template <>
struct Frag<bf16> {
  bf16x8 v;
  __device__ __forceinline__ void lds(const char* p) { v = *reinterpret_cast<const bf16x8*>(p); }
};
template <>
struct Frag<float> {
  float v[8];
  __device__ __forceinline__ void lds(const char* p) {
    float4 a = reinterpret_cast<const float4*>(p)[0];
    float4 b = reinterpret_cast<const float4*>(p)[1];
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
  }
};
__device__ __forceinline__ f32x4 mma(const Frag<bf16>& a, const Frag<bf16>& b, f32x4 c) {
  return __builtin_amdgcn_mfma_f32_16x16x32_bf16(a.v, b.v, c, 0, 0, 0);
}
__device__ __forceinline__ f32x4 mma(const Frag<float>& a, const Frag<float>& b, f32x4 c) {
  // k-slot h (= lane>>4) of MFMA j carries k = 8h + j: same map for A and B.
#pragma unroll
  for (int j = 0; j < 8; ++j) c = __builtin_amdgcn_mfma_f32_16x16x4f32(a.v[j], b.v[j], c, 0, 0, 0);
  return c;
}

// shared epilogue: bias [+ residual] -> BN partials -> [sigmoid] -> store (NHWC T or NCHW f32)
// STAGED (bf16 NHWC only): after bias and BN partials the tile is rounded to bf16, written
// to LDS (16-B chunks XOR-swizzled by pixel row) and stored with coalesced 16-B row
// segments; the residual (if any) is added in that pass.  smem must hold BM*BN*2 bytes.
// mid (persistent kernels): with a callable other than NoMid, every thread reads its store
// chunks back into registers, the block syncs (LDS free again) and mid() runs -- it issues
// the next tile's LDS-DMA prologue -- before the stores, which then drain under that DMA.
struct NoMid {
  __device__ void operator()() const {}
};
template <typename T, int WN, int WM, int RN, int RM, bool STAGED = false, typename Mid = NoMid>
__device__ __forceinline__ void conv_epilogue(const ConvArgs& a, f32x4 (&acc)[RN][RM], char* smem, int co0, int p0,
                                              int tm, int wn, int wm, int lane, int tid, Mid mid = Mid{}) {
  constexpr bool kMid = !std::is_same<Mid, NoMid>::value;
  constexpr int NT = 64 * WN * WM;
  constexpr int BN = WN * RN * 16;
  constexpr int BM = WM * RM * 16;
  const int HW = a.H * a.W;
  const int lr = lane & 15, lh = lane >> 4;
  // STAGED + residual: this thread's residual chunks of the store pass are loaded first, so
  // their HBM latency hides under the BN partials and the LDS staging (loaded inside the
  // store loop they were serialised behind its stores: +22 us per res conv at 64x64, B=32)
  constexpr int SCPR = BN / 8, NRES = STAGED ? (BM * SCPR + NT - 1) / NT : 1;
  uint4 rpre[NRES];
  // (with a mid hook the residual chunks are loaded after the LDS read-back instead, when the
  // accumulators are dead: their registers and the read-back's cannot all be live at once)
  auto load_res = [&]() {
    if (a.res) {
#pragma unroll
      for (int it = 0; it < NRES; ++it) {
        const int idx = tid + it * NT;
        const int pl = idx / SCPR, ch = idx - (idx / SCPR) * SCPR;
        const int tp = a.lgtw ? p0 + (pl >> a.lgtw) * a.W + (pl & ((1 << a.lgtw) - 1)) : p0 + pl;
        const int co = co0 + ch * 8;
        rpre[it] = make_uint4(0, 0, 0, 0);
        if (idx < BM * SCPR && tp < a.P && co < a.Cout)
          rpre[it] = *reinterpret_cast<const uint4*>(reinterpret_cast<const bf16*>(a.res) +
                                                      (long)out_pix(a, tp) * a.ldy + co);
      }
    }
  };
  if constexpr (STAGED && !kMid) load_res();
  float bv[RN][4];
#pragma unroll
  for (int n = 0; n < RN; ++n)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = co0 + wn * RN * 16 + n * 16 + lh * 4 + i;
      bv[n][i] = (a.bias && co < a.Cout) ? a.bias[co] : 0.f;
    }
  bool pv[RM];
  int pix_of[RM];
#pragma unroll
  for (int m = 0; m < RM; ++m) {
    const int loc = wm * RM * 16 + m * 16 + lr;
    const int tp = a.lgtw ? p0 + (loc >> a.lgtw) * a.W + (loc & ((1 << a.lgtw) - 1)) : p0 + loc;
    pv[m] = tp < a.P;
    pix_of[m] = out_pix(a, tp);
  }
#pragma unroll
  for (int n = 0; n < RN; ++n) {
    const int cb = co0 + wn * RN * 16 + n * 16 + lh * 4;
#pragma unroll
    for (int m = 0; m < RM; ++m) {
#pragma unroll
      for (int i = 0; i < 4; ++i) acc[n][m][i] += bv[n][i];
      if (!STAGED && a.res && pv[m]) {
        const T* rp = reinterpret_cast<const T*>(a.res) + (long)pix_of[m] * a.ldy + cb;
        if (cb + 3 < a.Cout) {
          float f[4];
          load4<T>(rp, f);
#pragma unroll
          for (int i = 0; i < 4; ++i) acc[n][m][i] += f[i];
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (cb + i < a.Cout) acc[n][m][i] += Elt<T>::to_f(rp[i]);
        }
      }
    }
  }

  // (records past cdiv(output pixels, RM*16) -- the empty wave rows of a partial last pixel
  // tile -- are not written: the caller sized the buffer with that many, fv_conv2d_stats_blocks;
  // the sub-pixel launches number records over the 4 phases of a low-res a.P, hence Ho x Wo)
  const long pout = a.Ho ? (long)a.N * a.Ho * a.Wo : (long)a.P;
  if (a.stats && (long)(tm * WM + wm) < (pout + RM * 16 - 1) / (RM * 16) && tm * WM + wm < a.nrec) {
    // BN statistics partials, one record per wave row (RM*16 pixels, record index
    // tm*WM + wm): per output channel (sum, sum of squares) over the record's valid pixels,
    // reduced over the 16 pixel lanes of each m-tile by shuffles -- no LDS, no barrier.
    const int rec = tm * WM + wm;
#pragma unroll
    for (int n = 0; n < RN; ++n) {
      float sv[4], qv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t = 0.f, q = 0.f;
#pragma unroll
        for (int m = 0; m < RM; ++m) {
          const float v = pv[m] ? acc[n][m][i] : 0.f;
          t += v;
          q += v * v;
        }
        sv[i] = row16_sum(t);
        qv[i] = row16_sum(q);
      }
      // every lane of a 16-lane row holds the row's 4 channel sums: lanes 0-3 store the sums,
      // lanes 4-7 the squares (one store instruction per n, 4 x 2 x 16 B)
      const int cb = co0 + wn * RN * 16 + n * 16 + lh * 4;
      const int ii = lr & 3;
      const float s01 = ii & 1 ? sv[1] : sv[0], s23 = ii & 1 ? sv[3] : sv[2];
      const float q01 = ii & 1 ? qv[1] : qv[0], q23 = ii & 1 ? qv[3] : qv[2];
      const float val = lr < 4 ? (ii & 2 ? s23 : s01) : (ii & 2 ? q23 : q01);
      if (lr < 8 && cb + ii < a.Cout) a.stats[(long)(rec * 2 + (lr >> 2)) * a.Cout + cb + ii] = val;
    }
  }

  if constexpr (STAGED) {
    static_assert(sizeof(T) == 2, "staged epilogue is bf16 NHWC");
    constexpr int CPR = BN / 8;                         // 16-B chunks per pixel row
    __syncthreads();                                    // stats scratch / last k-step reads done
#pragma unroll
    for (int n = 0; n < RN; ++n) {
      const int cl = wn * RN * 16 + n * 16 + lh * 4;    // local channel of this lane's 4 values
#pragma unroll
      for (int m = 0; m < RM; ++m) {
        const int pl = wm * RM * 16 + m * 16 + lr;
        bf16 t4[4] = {(bf16)acc[n][m][0], (bf16)acc[n][m][1], (bf16)acc[n][m][2], (bf16)acc[n][m][3]};
        char* dst = smem + pl * BN * 2 + (((cl >> 3) ^ (pl & (CPR - 1))) << 4) + ((cl & 4) << 1);
        *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(t4);
      }
    }
    __syncthreads();
    uint4 vv[kMid ? NRES : 1];
    if constexpr (kMid) {
#pragma unroll
      for (int it = 0; it < NRES; ++it) {
        const int idx = tid + it * NT;
        const int pl = idx / CPR, ch = idx - (idx / CPR) * CPR;
        if (idx < BM * CPR) vv[it] = *reinterpret_cast<const uint4*>(smem + pl * BN * 2 + ((ch ^ (pl & (CPR - 1))) << 4));
      }
      __syncthreads();
      load_res();
      mid();
    }
    auto chunk = [&](int it, int pl, int ch) -> uint4 {
      if constexpr (kMid) return vv[it];
      else return *reinterpret_cast<const uint4*>(smem + pl * BN * 2 + ((ch ^ (pl & (CPR - 1))) << 4));
    };
    if (!a.spm) {
      // the plain store pass (kept free of the record code below: +2-3 us per res conv)
#pragma unroll
      for (int it = 0; it < NRES; ++it) {
        const int idx = tid + it * NT;
        if (idx >= BM * CPR) break;
        const int pl = idx / CPR, ch = idx - (idx / CPR) * CPR;
        const int tp = a.lgtw ? p0 + (pl >> a.lgtw) * a.W + (pl & ((1 << a.lgtw) - 1)) : p0 + pl;
        const int co = co0 + ch * 8;
        if (tp >= a.P || co >= a.Cout) continue;
        const int pix = out_pix(a, tp);
        Chunk8<bf16> v;
        v.raw = chunk(it, pl, ch);
        T* yp = reinterpret_cast<T*>(a.y) + (long)pix * a.ldy + co;
        if (a.res) {
          Chunk8<bf16> r;
          r.raw = rpre[it];
          float f[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = v.get(j) + r.get(j);
          v.set8(f);
        }
        v.store(reinterpret_cast<bf16*>(yp));
      }
      return;
    }
    // store-pass records: NT % CPR == 0 keeps every thread on one 8-channel chunk for all its
    // iterations (the host enables spm only for such tiles, with P % BM == 0)
    const int sch = tid % CPR;
    float sacc[8], qacc[8], bm_[8], bi_[8], bg_[8], bb_[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) sacc[j] = qacc[j] = 0.f;
    if (a.spm == 2) {
      const int c = co0 + sch * 8;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const bool ok = c + j < a.Cout;
        bm_[j] = ok ? a.bnm[c + j] : 0.f;
        bi_[j] = ok ? a.bni[c + j] : 0.f;
        bg_[j] = ok ? a.bng[c + j] : 0.f;
        bb_[j] = ok ? a.bnb[c + j] : 0.f;
      }
    }
#pragma unroll
    for (int it = 0; it < NRES; ++it) {
      const int idx = tid + it * NT;
      if (idx >= BM * CPR) break;
      const int pl = idx / CPR, ch = idx - (idx / CPR) * CPR;
      const int tp = a.lgtw ? p0 + (pl >> a.lgtw) * a.W + (pl & ((1 << a.lgtw) - 1)) : p0 + pl;
      const int co = co0 + ch * 8;
      if (tp >= a.P || co >= a.Cout) continue;
      const int pix = out_pix(a, tp);
      Chunk8<bf16> v;
      v.raw = chunk(it, pl, ch);
      T* yp = reinterpret_cast<T*>(a.y) + (long)pix * a.ldy + co;
      Chunk8<bf16> r;
      r.raw = rpre[it];
      if (a.spm == 2) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float yh = (r.get(j) - bm_[j]) * bi_[j];
          const float gv = v.get(j);
          const float g = bg_[j] * yh + bb_[j] > 0.f ? gv : gv * a.bns;
          sacc[j] += g;
          qacc[j] += g * yh;
        }
      } else {
        if (a.res) {
          float f[8];
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = v.get(j) + r.get(j);
          v.set8(f);
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const float o = v.get(j);
          sacc[j] += o;
          qacc[j] += o * o;
        }
      }
      v.store(reinterpret_cast<bf16*>(yp));
    }
    {
      static_assert(CPR <= 64 && 64 % CPR == 0, "store-pass records: chunks per row must divide a wave");
#pragma unroll
      for (int o = CPR; o < 64; o <<= 1)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          sacc[j] += __shfl_xor(sacc[j], o, 64);
          qacc[j] += __shfl_xor(qacc[j], o, 64);
        }
      const int c = co0 + sch * 8;
      if (lane < CPR && c < a.Cout) {
        const long rec = (long)tm * (NT / 64) + (tid >> 6);
        float* r0 = a.sprec + (rec * 2) * a.Cout + c;
        float* r1 = a.sprec + (rec * 2 + 1) * a.Cout + c;
        *reinterpret_cast<float4*>(r0) = make_float4(sacc[0], sacc[1], sacc[2], sacc[3]);
        *reinterpret_cast<float4*>(r0 + 4) = make_float4(sacc[4], sacc[5], sacc[6], sacc[7]);
        *reinterpret_cast<float4*>(r1) = make_float4(qacc[0], qacc[1], qacc[2], qacc[3]);
        *reinterpret_cast<float4*>(r1 + 4) = make_float4(qacc[4], qacc[5], qacc[6], qacc[7]);
      }
    }
    return;
  }
#pragma unroll
  for (int n = 0; n < RN; ++n) {
    const int cb = co0 + wn * RN * 16 + n * 16 + lh * 4;
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      if (!pv[m]) continue;
      float f[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        f[i] = acc[n][m][i];
        if (a.sigmoid) f[i] = 1.f / (1.f + expf(-f[i]));
      }
      if (a.nchw) {
        float* yp = reinterpret_cast<float*>(a.y);
        const int img = pix_of[m] / HW, hw = pix_of[m] - img * HW;
#pragma unroll
        for (int i = 0; i < 4; ++i)
          if (cb + i < a.Cout) yp[((long)img * a.Cout + cb + i) * HW + hw] = f[i];
      } else {
        T* yp = reinterpret_cast<T*>(a.y) + (long)pix_of[m] * a.ldy + cb;
        if (cb + 3 < a.Cout) {
          store4<T>(yp, f);
        } else {
#pragma unroll
          for (int i = 0; i < 4; ++i)
            if (cb + i < a.Cout) yp[i] = Elt<T>::from_f(f[i]);
        }
      }
    }
  }
}

template <typename T, int KS, int WN, int WM, int RN, int RM, bool PRO, bool UPS>
__global__ void __launch_bounds__(64 * WN * WM)
conv_fwd_kernel(ConvArgs a) {
  constexpr int NT = 64 * WN * WM;
  constexpr int BN = WN * RN * 16;   // output channels per block
  constexpr int BM = WM * RM * 16;   // pixels per block
  constexpr int PAD = KS / 2;
  constexpr int ES = sizeof(T);
  constexpr int ROWB = BK * ES;
  constexpr int CA = BM * 4 / NT;
  constexpr int NBCH = BN * 4;
  constexpr int CB = (NBCH + NT - 1) / NT;
  static_assert((BM * 4) % NT == 0, "A staging");
  __shared__ __attribute__((aligned(16))) char smem[2 * (BM + BN) * ROWB];

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ wk = reinterpret_cast<const T*>(a.w);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wn = wave % WN, wm = wave / WN;
  const int tn = blockIdx.x % a.ntn, tm = blockIdx.x / a.ntn;
  const int co0 = tn * BN, p0 = tm * BM;
  const int kc = tid & 3;
  const int HW = a.H * a.W;

  int rh[CA], rw[CA], rb[CA];
  bool rv[CA];
#pragma unroll
  for (int i = 0; i < CA; ++i) {
    const int pix = p0 + (tid >> 2) + i * (NT / 4);
    rv[i] = pix < a.P;
    const int n = pix / HW;
    const int rem = pix - n * HW;
    rh[i] = rem / a.W;
    rw[i] = rem - rh[i] * a.W;
    rb[i] = n * a.Hin * a.Win;
  }

  Chunk8<T> ra[CA], rbw[CB];
  unsigned okm = 0;
  int cur_ci = 0;

  auto gload = [&](int ks) {
    const int k = ks * BK + kc * 8;
    const bool kin = k < a.K;
    const int tap = k >> a.lgCin;
    const int ci = k & (a.Cin - 1);
    const int r = tap / KS, s = tap - (tap / KS) * KS;
    cur_ci = ci;
    okm = 0;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int hh = rh[i] + r - PAD, ww = rw[i] + s - PAD;
      bool ok = kin && rv[i];
      int hs, ws;
      if constexpr (UPS) {
        ok = ok && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
        hs = hh >> 1;
        ws = ww >> 1;
      } else {
        ok = ok && hh >= 0 && hh < a.Hin && ww >= 0 && ww < a.Win;
        hs = hh;
        ws = ww;
      }
      if (ok) {
        ra[i].load(x + ((long)(rb[i] + hs * a.Win + ws) << a.lgCin) + ci);
        okm |= 1u << i;
      } else {
        ra[i].zero();
      }
    }
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const int q = tid + j * NT;
      if (q < NBCH) rbw[j].load(wk + (long)(co0 + (q >> 2)) * a.Kpad + ks * BK + kc * 8);
    }
  };

  auto lstore = [&](int buf) {
    char* As = smem + buf * (BM + BN) * ROWB;
    char* Bs = As + BM * ROWB;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int row = (tid >> 2) + i * (NT / 4);
      Chunk8<T> c = ra[i];
      if constexpr (PRO) {
        if (okm & (1u << i)) {
          float f[8];
          const float4 s0 = *reinterpret_cast<const float4*>(a.psc + cur_ci);
          const float4 s1 = *reinterpret_cast<const float4*>(a.psc + cur_ci + 4);
          const float4 h0 = *reinterpret_cast<const float4*>(a.psh + cur_ci);
          const float4 h1 = *reinterpret_cast<const float4*>(a.psh + cur_ci + 4);
          const float sc[8] = {s0.x, s0.y, s0.z, s0.w, s1.x, s1.y, s1.z, s1.w};
          const float sh[8] = {h0.x, h0.y, h0.z, h0.w, h1.x, h1.y, h1.z, h1.w};
#pragma unroll
          for (int j = 0; j < 8; ++j) f[j] = fv_act(c.get(j) * sc[j] + sh[j], a.slope);
          c.set8(f);
        }
      }
      c.store(reinterpret_cast<T*>(As + row * ROWB + ((kc ^ rswz<T>(row)) * 8 * ES)));
    }
#pragma unroll
    for (int j = 0; j < CB; ++j) {
      const int q = tid + j * NT;
      if (q < NBCH) {
        const int row = q >> 2;
        rbw[j].store(reinterpret_cast<T*>(Bs + row * ROWB + ((kc ^ rswz<T>(row)) * 8 * ES)));
      }
    }
  };

  f32x4 acc[RN][RM];
#pragma unroll
  for (int n = 0; n < RN; ++n)
#pragma unroll
    for (int m = 0; m < RM; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lh = lane >> 4;
  auto compute = [&](int buf) {
    const char* As = smem + buf * (BM + BN) * ROWB;
    const char* Bs = As + BM * ROWB;
    Frag<T> af[RN], bfm[RM];
#pragma unroll
    for (int n = 0; n < RN; ++n) {
      const int row = wn * RN * 16 + n * 16 + lr;
      af[n].lds(Bs + row * ROWB + ((lh ^ rswz<T>(row)) * 8 * ES));
    }
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int row = wm * RM * 16 + m * 16 + lr;
      bfm[m].lds(As + row * ROWB + ((lh ^ rswz<T>(row)) * 8 * ES));
    }
#pragma unroll
    for (int n = 0; n < RN; ++n)
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[n][m] = mma(af[n], bfm[m], acc[n][m]);
  };

  gload(0);
  lstore(0);
  __syncthreads();
  for (int ks = 0; ks < a.nks; ++ks) {
    const int cur = ks & 1;
    if (ks + 1 < a.nks) gload(ks + 1);
    compute(cur);
    if (ks + 1 < a.nks) lstore(cur ^ 1);
    __syncthreads();
  }

  conv_epilogue<T, WN, WM, RN, RM>(a, acc, smem, co0, p0, tm, wn, wm, lane, tid);
}

// ----------------------------------------------------------------------------------------
// v2 forward (bf16, cin % 64 == 0): both operands land in LDS by DMA (buffer/global_load
// ... lds, no VGPR staging, no ds_write), BK = 64 (one tap x 64 channels per step), 128-B
// rows XOR-swizzled through the SOURCE address (the DMA destination is lane-linear),
// double-buffered with one barrier per step.  Zero padding comes from the buffer range
// check: an out-of-image tap gets voffset >= num_records and the hardware returns 0.
// ----------------------------------------------------------------------------------------
constexpr int BK2 = 64;
__device__ __forceinline__ int swz8(int row) { return (row >> 1) & 7; }

typedef __attribute__((address_space(3))) void* lds_ptr_t;

// 16 B per lane, buffer -> LDS (wave-uniform LDS byte address in M0, lane-linear
// destination), byte offset voffset + soffset (an out-of-range voffset of 0x80000000 stays
// out of range for any soffset < 2^31, so the hardware returns zeros).
// Issued as inline asm on purpose: hipcc cannot tell that the ds_reads of the buffer being
// computed do not alias the stage in flight and would put an s_waitcnt vmcnt(0) in front
// of them, serialising the ring.  Ordering is therefore explicit: counted vmcnt + barrier.
// The asm has NO outputs (M0 is declared clobbered): hipcc models an inline asm containing a
// VMEM op as writing its outputs asynchronously and waits vmcnt(0) before such a register is
// reused -- with an output, every DMA of a loop waited for the previous one.
// lgkmcnt(0) as the s_waitcnt builtin, not inline asm: the compiler's wait-count pass sees it
// and knows every LDS read issued before it has landed.  After an inline-asm wait the pass
// still counts those reads as outstanding, and with more than 15 reads in flight (the 4-bit
// lgkm counter) it waits for the NEWEST reads before the first use of an old fragment: in
// the pair-of-taps loops every step's second MFMA cluster waited for the next tap's 12
// fragment reads (lgkmcnt(7) .. (0) in front of its first 8 MFMAs).
__device__ __forceinline__ void wait_lgkm0() {
  asm volatile("" ::: "memory");
  __builtin_amdgcn_s_waitcnt(0xC07F);       // vmcnt(63) expcnt(7) lgkmcnt(0)
}

__device__ __forceinline__ void dma16s(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff, unsigned soff) {
  // lds / soff are wave-uniform at every call site (the "s" operands); readfirstlane states it
  // for values the compiler merges across uniform branches into a VGPR phi (a no-op on an SGPR)
  lds = __builtin_amdgcn_readfirstlane(lds);
  soff = __builtin_amdgcn_readfirstlane(soff);
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, %3 offen lds"
               :
               : "v"(voff), "s"(r), "s"(lds), "s"(soff)
               : "memory", "m0");
}
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t r, const void* lds, unsigned voff) {
  dma16s(r, __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)lds), voff, 0u);
}

// f(integral_constant<S>) for the run-time, wave-uniform s in [0, N): a scalar branch to
// one of N instantiations, so register arrays are only ever indexed by constants
template <int S, int N, typename F>
__device__ __forceinline__ void with_const(int s, F&& f) {
  if constexpr (S + 1 == N) {
    f(std::integral_constant<int, S>{});
  } else {
    if (s == S) f(std::integral_constant<int, S>{});
    else with_const<S + 1, N>(s, f);
  }
}

// BKS = k per stage: 64 (128-B rows, 8 chunks) or 32 (64-B rows, 4 chunks; half the LDS, so
// the 4-wave tiles run 4 blocks per CU and hide each other's DMA latency and epilogue).
template <int BKS>
__device__ __forceinline__ int swzk(int row) {
  if constexpr (BKS == 64) return swz8(row);
  else return rswz<bf16>(row);
}

// MODE 0: plain conv; 1: nearest-x2 upsample folded into the addressing (tile space =
// output); 2: one sub-pixel phase of an upsample + 3x3 conv = a 2x2 conv over the low-res
// input with phase-folded weights (tile space = low-res image, block phase = lid & 3,
// KS == 2, taps at offsets {-1, 0} or {0, +1} per phase coordinate); 3: stride-2 4x4 conv
// (input coordinate 2 * out + tap - 1): the data gradient of an upsample + 3x3 conv
// straight at the low resolution (tile space = low-res dx, input = high-res dy).
template <int KS, int WN, int WM, int RN, int RM, int MODE, int BKS>
__global__ void __launch_bounds__(64 * WN * WM, (BKS == 32 && WN * WM == 4) ? 4 : 2)
conv_fwd_v2(ConvArgs a, unsigned x_bytes) {
  constexpr bool UPS = MODE == 1;
  constexpr int NW = WN * WM;
  constexpr int BN = WN * RN * 16, BM = WM * RM * 16;
  constexpr int PAD = KS / 2;
  constexpr int ROWB = BKS * 2;
  constexpr int CH = BKS / 8, RPP = 64 / CH;         // 16-B chunks per row, rows per 1-KB piece
  constexpr int QA = BM / RPP, QB = BN / RPP;        // 1-KB DMA pieces per stage
  constexpr int JA = (QA + NW - 1) / NW, JB = (QB + NW - 1) / NW;
  constexpr int STAGE = (BM + BN) * ROWB;
  __shared__ __attribute__((aligned(1024))) char smem[2 * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int nks = a.nks * (64 / BKS);   // a.nks counts 64-deep steps
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wm = wave / WN;
  // XCD-aware tile order: blocks b, b+8, ... share an XCD (observed round-robin dispatch);
  // give each XCD a contiguous run of logical tiles (co tiles of a pixel tile, then its
  // neighbours, which share halo rows).  Bijective for any grid size.  Speed only.
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int lid0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  // MODE 2: the 4 phases of one low-res tile are neighbours (same input rows)
  const int phase = MODE == 2 ? (lid0 & 3) : 0;
  const int lid = MODE == 2 ? (lid0 >> 2) : lid0;
  if constexpr (MODE == 2) a.sub = 1 + phase;
  const int pa = phase >> 1, pb = phase & 1;
  // row / column tap offset: centred (MODE 0/1), per phase (MODE 2), -1 after the stride (3)
  const int roff = MODE == 2 ? pa - 1 : MODE == 3 ? -1 : -PAD;
  const int coff = MODE == 2 ? pb - 1 : MODE == 3 ? -1 : -PAD;
  constexpr int STR = MODE == 3 ? 2 : 1;
  const int tn = lid % a.ntn, tm = lid / a.ntn;
  const int co0 = tn * BN, p0 = tm * BM;
  const int HW = a.H * a.W;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7fffffff, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);
  const int lrow = lane / CH, lchk = lane % CH;
  // per-piece constants.  A piece is RPP consecutive pixels of ONE image row (W % RPP == 0,
  // so p0 + RPP*q never straddles a row) x CH 16-B chunks: its image row (n, h) is wave-uniform and
  // the row part of the source address goes to soffset (SALU only); the lane's column part
  // for each tap column s is precomputed once, 0x80000000 marking a column outside the
  // image (the buffer range check then returns 0).  A k-step costs no address VALU beyond
  // selecting the tap column's register.
  int prn[JA], prh[JA];
  bool pok[JA];
  unsigned vcol[JA][KS];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int q = wave + j * NW;
    const int pp = __builtin_amdgcn_readfirstlane(p0 + q * RPP);
    pok[j] = (QA % NW == 0 || q < QA) && pp < a.P;
    const int n = pp / HW, rem = pp - n * HW;
    const int h = rem / a.W, w0 = rem - h * a.W;
    prn[j] = n * a.Hin;
    prh[j] = h;
    const unsigned chunk = (unsigned)((lchk ^ swzk<BKS>(q * RPP + lrow)) << 3);
#pragma unroll
    for (int s = 0; s < KS; ++s) {
      const int ww = STR * (w0 + lrow) + s + coff;
      const int sc = UPS ? (ww >> 1) : ww;
      const int wlim = UPS ? a.W : a.Win;
      vcol[j][s] = (ww >= 0 && ww < wlim) ? ((unsigned)(sc << a.lgCin) + chunk) * 2u : 0x80000000u;
    }
  }
  unsigned wbase[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int row = (wave + j * NW) * RPP + lrow;
    wbase[j] = (unsigned)(((co0 + row) * a.Kpad + ((lchk ^ swzk<BKS>(row)) << 3)) * 2);
  }

  auto issue = [&](int ks, int buf) {
    const int k0 = ks * BKS;
    const unsigned As = sbase + buf * STAGE;
    const unsigned Bs = As + BM * ROWB;
    const int tap = k0 >> a.lgCin, ci0 = k0 & (a.Cin - 1);
    const int r = tap / KS, s = tap - (tap / KS) * KS;
    with_const<0, KS>(s, [&](auto sc) {
      constexpr int S = decltype(sc)::value;
#pragma unroll
      for (int j = 0; j < JA; ++j) {
        const int q = wave + j * NW;
        if (QA % NW == 0 || q < QA) {
          const int hh = STR * prh[j] + r + roff;
          const int srow = UPS ? (hh >> 1) : hh;
          if (pok[j] && hh >= 0 && hh < (UPS ? a.H : a.Hin))
            dma16s(xr, As + q * 1024, vcol[j][S], (unsigned)((((prn[j] + srow) * a.Win) << a.lgCin) + ci0) * 2u);
          else
            dma16s(xr, As + q * 1024, 0x80000000u, 0u);
        }
      }
    });
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int q = wave + j * NW;
      if (QB % NW == 0 || q < QB) dma16s(wr, Bs + q * 1024, wbase[j], (unsigned)((k0 + phase * a.wphase) * 2));
    }
  };

  f32x4 acc[RN][RM];
#pragma unroll
  for (int n = 0; n < RN; ++n)
#pragma unroll
    for (int m = 0; m < RM; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int lr = lane & 15, lh = lane >> 4;
  // fragments of one 32-deep k half-step (kk) of LDS buffer `buf`
  auto load_frags = [&](Frag<bf16> (&fa)[RN], Frag<bf16> (&fb)[RM], int buf, int kk) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + BM * ROWB;
#pragma unroll
    for (int n = 0; n < RN; ++n) {
      const int row = wn * RN * 16 + n * 16 + lr;
      fa[n].lds(Bs + row * ROWB + (((kk * 4 + lh) ^ swzk<BKS>(row)) << 4));
    }
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int row = wm * RM * 16 + m * 16 + lr;
      fb[m].lds(As + row * ROWB + (((kk * 4 + lh) ^ swzk<BKS>(row)) << 4));
    }
  };
  // s_setprio(1) around each MFMA cluster keeps hipcc from moving MFMAs across the raw
  // barriers into the DMA / fragment-read sections (guide T5)
  constexpr bool prio = true;
  auto mfma_all = [&](const Frag<bf16> (&fa)[RN], const Frag<bf16> (&fb)[RM]) {
    if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int n = 0; n < RN; ++n)
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[n][m] = mma(fa[n], fb[m], acc[n][m]);
    if (prio) __builtin_amdgcn_s_setprio(0);
  };

  if (BKS == 64) {
    // Software-pipelined k loop: the fragments of the next half-step are read while the
    // MFMAs of the current one run, and the per-step barrier sits between the two MFMA
    // groups of a step, so after it the matrix pipe has the second group (already in
    // registers) to work on while the next step's first fragments and DMAs are issued.
    //   step ks:  read F1(ks) | MFMA F0(ks) | vmcnt(0)+lgkmcnt(0), barrier | DMA ks+2 -> buf,
    //             read F0(ks+1) | MFMA F1(ks)
    // The barrier publishes stage ks+1 (every wave waited for its own DMAs) and retires all
    // reads of buffer ks&1 (each wave drained its reads first), which DMA ks+2 then refills.
    Frag<bf16> fa0[RN], fb0[RM], fa1[RN], fb1[RM];
    issue(0, 0);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    if (nks > 1) issue(1, 1);
    load_frags(fa0, fb0, 0, 0);
    // steady state without branches around the fragment reads (a read on one path only
    // makes the compiler drain every LDS read before the next MFMA group)
    for (int ks = 0; ks + 1 < nks; ++ks) {
      const int buf = ks & 1;
      load_frags(fa1, fb1, buf, 1);
      mfma_all(fa0, fb0);
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (ks + 2 < nks) issue(ks + 2, buf);
      load_frags(fa0, fb0, buf ^ 1, 0);
      mfma_all(fa1, fb1);
    }
    load_frags(fa1, fb1, (nks - 1) & 1, 1);
    mfma_all(fa0, fb0);
    mfma_all(fa1, fb1);
  } else {
    // one barrier per step, fragments read per 32-deep half-step (the BKS = 32 loop)
    issue(0, 0);
    for (int ks = 0; ks < nks; ++ks) {
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
      __syncthreads();
      if (ks + 1 < nks) issue(ks + 1, (ks + 1) & 1);
#pragma unroll
      for (int kk = 0; kk < BKS / 32; ++kk) {
        Frag<bf16> af[RN], bfm[RM];
        load_frags(af, bfm, ks & 1, kk);
        mfma_all(af, bfm);
      }
    }
  }
  __syncthreads();
  conv_epilogue<bf16, WN, WM, RN, RM, true>(a, acc, smem, co0, p0, MODE == 2 ? tm * 4 + phase : tm, wn, wm, lane,
                                             tid);
}

// ----------------------------------------------------------------------------------------
// 3x3 stride-1 conv with a halo-staged input (bf16 NHWC, cin % 64 == 0, W % 64 == 0):
// the res / down convs and their data gradients.  The per-tap DMA of conv_fwd_v2 moves 9
// copies of every input pixel into LDS; at 1 KB per ~30 CU-cycles that fill, not the MFMA,
// bounds the short-K layers (AFE.down1 forward: DMA alone 300 us of 530).  Here a block owns
// TR = 4 image rows x 64 columns; per 32-channel chunk the (TR+2) x 66 halo lands in LDS once
// and the 9 taps read their shifted windows from it, so a 32-deep k step moves the weight
// slice (BN x 64 B) plus 1/9 of a halo: 1.7x (BN 256) to 2.6x (BN 64) fewer bytes per MAC.
//   k step ks = (chunk c = ks / 9, tap t = ks % 9); weights [co][tap][ci] as in v2.
//   halo pixel hp = hr * 66 + hc at hp * 64 B, 16-B chunk XOR ((hp >> 2) & 1) * 2: a fragment
//   read (16 consecutive halo pixels from ANY start) is bank-conflict free (ds_read_b128
//   lane groups of the guide's table).
// ----------------------------------------------------------------------------------------
__device__ __forceinline__ int h3swz(int hp) { return ((hp >> 2) & 1) << 1; }

template <int N>
__device__ __forceinline__ void wait_vm() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }
// wave-uniform count -> the matching immediate (counts above 15 wait for 15: stricter, safe)
__device__ __forceinline__ void wait_vm_dyn(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    case 8: wait_vm<8>(); break;
    case 9: wait_vm<9>(); break;
    case 10: wait_vm<10>(); break;
    case 11: wait_vm<11>(); break;
    case 12: wait_vm<12>(); break;
    case 13: wait_vm<13>(); break;
    case 14: wait_vm<14>(); break;
    default: wait_vm<15>(); break;
  }
}

// wave-uniform count 0 .. 63 (gfx950's vmcnt range) -> the matching immediate
template <int N = 63>
__device__ __forceinline__ void wait_vm_upto(int n) {
  if constexpr (N == 0) {
    wait_vm<0>();
  } else {
    if (n >= N) wait_vm<N>();
    else wait_vm_upto<N - 1>(n);
  }
}

// Software-pipelined variant: a step is a PAIR of taps (64 k), the weight stage holds both
// taps' 32-channel slices, and the loop is conv_fwd_v2's: the fragments of the step's second
// tap are read while the first tap's MFMAs run and the barrier sits between the two MFMA
// groups.  Chunk c's halo goes into buffer c & 1 right after the barrier that retires the
// last read of chunk c - 2 (5 steps before its first use).  The weight stages form a ring of
// NSB buffers issued NSB - 1 steps ahead, so a DMA has NSB - 2 full steps to land.
template <int WN, int WM, int RN, int RM, int NSB>
__global__ void __launch_bounds__(64 * WN * WM, WN * RN * 16 >= 256 ? 1 : 2)
conv3_halo_fwd2(ConvArgs a, unsigned x_bytes) {
  constexpr int NW = WN * WM;
  constexpr int BN = WN * RN * 16, BM = WM * RM * 16, TR = BM / 64;
  constexpr int HP = (TR + 2) * 66, HQ = (HP + 15) / 16, JH = (HQ + NW - 1) / NW;
  constexpr int HALO = HQ * 1024;
  constexpr int QB = BN / 16, JB = QB / NW;
  static_assert(QB % NW == 0, "weight pieces per wave");
  constexpr int BST = BN * 64, STG = 2 * BST;
  constexpr int MAIN = 2 * HALO + NSB * STG, EPI = BM * BN * 2;
  __shared__ __attribute__((aligned(1024))) char smem[MAIN > EPI ? MAIN : EPI];

  FV_DIAG_BEGIN();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tn = lid % a.ntn, tm = lid / a.ntn;
  const int tiles_w = a.W >> 6, tiles_h = a.H / TR;
  const int tw = tm % tiles_w, th = (tm / tiles_w) % tiles_h, n = tm / (tiles_w * tiles_h);
  const int co0 = tn * BN;
  const int p0 = (n * a.H + th * TR) * a.W + tw * 64;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7fffffff, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);
  const int lrow = lane >> 2, lchk = lane & 3;

  unsigned hoff[JH];
#pragma unroll
  for (int j = 0; j < JH; ++j) {
    const int hp = (wave + j * NW) * 16 + lrow;
    const int hr = hp / 66, hc = hp - (hp / 66) * 66;
    const int ih = th * TR + hr - 1, iw = tw * 64 + hc - 1;
    const bool ok = hp < HP && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
    hoff[j] = ok ? (unsigned)(((((n * a.H + ih) * a.W + iw) << a.lgCin) + ((lchk ^ h3swz(hp)) << 3)) * 2) : 0x80000000u;
  }
  // stage-major weights (weight_prep_body smaj, as conv3_halo_fwd3): piece jb of tap unit u is
  // the contiguous KB at u * ustep + (co0 + (wave + jb * NW) * 16) * 64
  unsigned wbase[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int row = (wave + j * NW) * 16 + lrow;
    wbase[j] = (unsigned)((co0 + row) * 64 + ((lchk ^ rswz<bf16>(row)) << 4));
  }
  const unsigned ustep = (unsigned)a.wus;
  const int nch = a.Cin >> 5, ntap = 9 * nch, nsteps = (ntap + 1) >> 1;
  auto issue_b = [&](int j, int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = 2 * j + h;
      if (u < ntap) {
        const unsigned Bs = sbase + 2 * HALO + buf * STG + h * BST;
#pragma unroll
        for (int jb = 0; jb < JB; ++jb) dma16s(wr, Bs + (wave + jb * NW) * 1024, wbase[jb], (unsigned)u * ustep);
      }
    }
  };
  auto issue_halo = [&](int c) {
    const unsigned Hs = sbase + (c & 1) * HALO;
#pragma unroll
    for (int j = 0; j < JH; ++j)
      if (j < JH - 1 || wave + j * NW < HQ) dma16s(xr, Hs + (wave + j * NW) * 1024, hoff[j], (unsigned)(c * 64));
  };

  const int lr = lane & 15, lh = lane >> 4;
  int hpb[RM];
#pragma unroll
  for (int m = 0; m < RM; ++m) {
    const int loc = wm * RM * 16 + m * 16 + lr;
    hpb[m] = (loc >> 6) * 66 + (loc & 63);
  }
  auto load_frags = [&](Frag<bf16> (&fa)[RN], Frag<bf16> (&fb)[RM], int u, int buf) {
    const int c = u / 9, t = u - c * 9, r = t / 3, s3 = t - (t / 3) * 3;
    const char* Bs = smem + 2 * HALO + buf * STG + (u & 1) * BST;
    const char* Hs = smem + (c & 1) * HALO;
#pragma unroll
    for (int i = 0; i < RN; ++i) {
      const int row = wn * RN * 16 + i * 16 + lr;
      fa[i].lds(Bs + row * 64 + ((lh ^ rswz<bf16>(row)) << 4));
    }
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int hp = hpb[m] + r * 66 + s3;
      fb[m].lds(Hs + hp * 64 + ((lh ^ h3swz(hp)) << 4));
    }
  };
  f32x4 acc[RN][RM];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int m = 0; m < RM; ++m) acc[i][m] = f32x4{0.f, 0.f, 0.f, 0.f};
  constexpr bool prio = true;
  auto mfma_all = [&](const Frag<bf16> (&fa)[RN], const Frag<bf16> (&fb)[RM]) {
    if (prio) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[i][m] = mma(fa[i], fb[m], acc[i][m]);
    if (prio) __builtin_amdgcn_s_setprio(0);
  };

  Frag<bf16> fa0[RN], fb0[RM], fa1[RN], fb1[RM];
  auto bcnt = [&](int j) { return j < nsteps ? (2 * j + 1 < ntap ? 2 : 1) * JB : 0; };
  // ring of NSB weight stages: stage j in buffer j % NSB, issued NSB - 1 steps ahead; the
  // barrier of step j waits for stage j + 1 only (counted vmcnt: what this wave issued in
  // step j - 1 may stay in flight)
  issue_b(0, 0);
  issue_halo(0);
  if (nch > 1) issue_halo(1);
  for (int i = 1; i < NSB - 1; ++i)
    if (i < nsteps) issue_b(i, i);
  wait_vm<0>();
  __syncthreads();
  FV_DIAG_PROLOGUE();
  int pend = 0;                                 // DMAs this wave issued in the previous step
  if (NSB - 1 < nsteps) {
    issue_b(NSB - 1, NSB - 1);
    pend = bcnt(NSB - 1);
  }
  load_frags(fa0, fb0, 0, 0);
  int hn = 2, hstep = (9 * 2 - 10) / 2;         // next halo chunk and the step that issues it
  int bj = 0;                                   // buffer of stage j
  // No branch around the fragment reads: a read issued on one path only makes the compiler
  // drain ALL LDS reads (lgkmcnt(0)) before the next MFMA group, exposing the F1 read latency
  // every step.  An odd last tap re-reads a valid tap and skips its MFMAs.
  // The last step is peeled (its odd tap, if any, re-reads a valid tap and skips the MFMAs):
  // inside the loop its path (no barrier, no next-tap reads) merged into the loop's second
  // MFMA cluster and made the wait-count pass hold that cluster for the next tap's reads.
  for (int j = 0; j + 1 < nsteps; ++j) {
    load_frags(fa1, fb1, 2 * j + 1, bj);
    mfma_all(fa0, fb0);
    const int bn1 = bj + 1 == NSB ? 0 : bj + 1;
    // the weight stage is issued LAST in a step, so the count left in flight is that
    // stage's alone (a halo issued before it is waited for one step later)
    FV_DIAG_WAIT_BEGIN();
    if constexpr (NSB == 2) wait_vm<0>();     // stage j + 1 was the one issued last
    else if (pend == 2 * JB) wait_vm<2 * JB>();
    else wait_vm_dyn(pend);
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    FV_DIAG_WAIT_END();
    if (hn < nch && j == hstep) {
      issue_halo(hn);
      ++hn;
      hstep = (9 * hn - 10) / 2;
    }
    pend = 0;
    if (j + NSB < nsteps) {
      issue_b(j + NSB, bj);
      pend = bcnt(j + NSB);
    }
    load_frags(fa0, fb0, 2 * j + 2, bn1);
    FV_DIAG_ISSUE_END();
    mfma_all(fa1, fb1);
    bj = bn1;
  }
  {
    const int j = nsteps - 1;
    const bool two = 2 * j + 1 < ntap;
    load_frags(fa1, fb1, two ? 2 * j + 1 : 2 * j, bj);
    mfma_all(fa0, fb0);
    if (two) mfma_all(fa1, fb1);
  }
  FV_DIAG_LOOP_END();
  __syncthreads();
  conv_epilogue<bf16, WN, WM, RN, RM, true>(a, acc, smem, co0, p0, tm, wn, wm, lane, tid);
  FV_DIAG_END();
}

// Epilogue of conv3_halo_fwd3 MODE 1 (sub-pixel forward): tile columns are 4 phases x 64
// channels (wave column wn = phase (pa, pb)), rows the 256 low-res pixels (h0 + r, w0 + col).
// bias -> BN records -> bf16 through LDS -> 16-B stores to output pixel (2h + pa, 2w + pb).
// BN records: one per (tile, wave row, phase) = RM * 16 output pixels, record index
// ((tm * WM + wm) * 4 + wn) (stats_record_pixels: 128), so every output pixel is in one record.
template <int WM, int RM, typename Mid = NoMid>
__device__ __forceinline__ void subpix_epilogue(const ConvArgs& a, f32x4 (&acc)[4][RM], char* smem, int tn, int n,
                                                int h0, int w0, int tm, int wn, int wm, int lane, int tid,
                                                Mid mid = Mid{}) {
  constexpr bool kMid = !std::is_same<Mid, NoMid>::value;
  constexpr int RN = 4, NT = 64 * 4 * WM, BN = 256, BM = WM * RM * 16, CPR = BN / 8;
  const int lr = lane & 15, lh = lane >> 4;
  const int cb0 = tn * 64;
#pragma unroll
  for (int nn = 0; nn < RN; ++nn)
#pragma unroll
    for (int i = 0; i < 4; ++i) {
      const int co = cb0 + nn * 16 + lh * 4 + i;
      const float bv = a.bias ? a.bias[co] : 0.f;
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[nn][m][i] += bv;
    }
  if (a.stats) {
    const int rec = (tm * WM + wm) * 4 + wn;
#pragma unroll
    for (int nn = 0; nn < RN; ++nn) {
      float sv[4], qv[4];
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        float t = 0.f, q = 0.f;
#pragma unroll
        for (int m = 0; m < RM; ++m) {
          t += acc[nn][m][i];
          q += acc[nn][m][i] * acc[nn][m][i];
        }
        sv[i] = row16_sum(t);
        qv[i] = row16_sum(q);
      }
      const int cb = cb0 + nn * 16 + lh * 4;
      const int ii = lr & 3;
      const float s01 = ii & 1 ? sv[1] : sv[0], s23 = ii & 1 ? sv[3] : sv[2];
      const float q01 = ii & 1 ? qv[1] : qv[0], q23 = ii & 1 ? qv[3] : qv[2];
      const float val = lr < 4 ? (ii & 2 ? s23 : s01) : (ii & 2 ? q23 : q01);
      if (lr < 8 && rec < a.nrec) a.stats[(long)(rec * 2 + (lr >> 2)) * a.Cout + cb + ii] = val;
    }
  }
  __syncthreads();
#pragma unroll
  for (int nn = 0; nn < RN; ++nn) {
    const int cl = wn * 64 + nn * 16 + lh * 4;
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int pl = wm * RM * 16 + m * 16 + lr;
      bf16 t4[4] = {(bf16)acc[nn][m][0], (bf16)acc[nn][m][1], (bf16)acc[nn][m][2], (bf16)acc[nn][m][3]};
      char* dst = smem + pl * BN * 2 + (((cl >> 3) ^ (pl & (CPR - 1))) << 4) + ((cl & 4) << 1);
      *reinterpret_cast<uint2*>(dst) = *reinterpret_cast<const uint2*>(t4);
    }
  }
  __syncthreads();
  constexpr int NIT = BM * CPR / NT;
  static_assert(BM * CPR % NT == 0, "store pass");
  uint4 vv[kMid ? NIT : 1];
  if constexpr (kMid) {
#pragma unroll
    for (int it = 0; it < NIT; ++it) {
      const int idx = tid + it * NT;
      const int pl = idx / CPR, ch = idx - (idx / CPR) * CPR;
      vv[it] = *reinterpret_cast<const uint4*>(smem + pl * BN * 2 + ((ch ^ (pl & (CPR - 1))) << 4));
    }
    __syncthreads();
    mid();
  }
#pragma unroll
  for (int it = 0; it < NIT; ++it) {
    const int idx = tid + it * NT;
    const int pl = idx / CPR, ch = idx - (idx / CPR) * CPR;
    const int ph = ch >> 3, co = cb0 + (ch & 7) * 8;
    const int oh = 2 * (h0 + (pl >> 6)) + (ph >> 1), ow = 2 * (w0 + (pl & 63)) + (ph & 1);
    Chunk8<bf16> v;
    if constexpr (kMid) v.raw = vv[it];
    else v.raw = *reinterpret_cast<const uint4*>(smem + pl * BN * 2 + ((ch ^ (pl & (CPR - 1))) << 4));
    v.store(reinterpret_cast<bf16*>(a.y) + ((long)(n * a.Ho + oh) * a.Wo + ow) * a.ldy + co);
  }
}

// Linear-halo variant of conv3_halo_fwd2: every LDS fragment address is a per-lane base
// register plus an immediate.  In fwd2 the XOR swizzle of a 64-B halo pixel moves with the tap
// shift, so each of the 16 fragment reads of a step costs ~5 VALU (88 non-MFMA VALU per 64
// MFMAs): with two waves per SIMD that fills most of the vector issue slots the MFMAs leave.
// Here a halo pixel takes 96 B (64 B of channels + 32 B zero-filled by out-of-range DMA
// slots): 16 consecutive pixels read by ds_read_b128 from ANY start are conflict-free, and the
// address of pixel hp shifted by a tap is linear: a tap adds one wave-uniform offset to a
// per-lane base and the fragments of the step are immediate offsets from it (measured in the
// asm: 4 non-MFMA VALU per 64-MFMA step against 88).  LDS: [NSB weight stages][2 halo buffers].
//
// SCH (schedule of the two waves of a SIMD, waves w and w + NW / 2): bit 0 = one static
// s_setprio 1 for waves NW/2 .. NW-1 before the main loop instead of prio flips around every
// MFMA cluster; bit 1 = stagger: waves NW/2 .. NW-1 pass each step's barrier before the MFMAs
// of the tap whose fragments they hold, so they run those MFMAs while their partners issue the
// DMA and fragment reads after the barrier, and issue their own reads while the partners run
// MFMAs (same arithmetic, same order per accumulator: bit-identical).
//
// MODE (UpBlock2D's nearest-x2 upsample + 3x3 conv, modules.py:78-89, on this kernel's halo
// structure; the sub-pixel algebra of conv_fwd_v2 MODE 2 / 3):
//   1 = sub-pixel forward over the LOW-res input: the 256-row co tile is 4 phases (pa, pb) x 64
//       channels, wave column wn = phase; a 32-channel chunk has 4 tap units q = (rr, ss), the
//       phase's 2x2 folded taps, which read the halo window tap (pa + rr, pb + ss); the
//       epilogue stores phase wn of low-res pixel (h, w) to output pixel (2h + pa, 2w + pb).
//   2 = data gradient at the LOW resolution: dy viewed as 4 phase planes (py, px) of the low-res
//       grid, the conv input = [plane][Cout] channels (a.Cin = 4 Cout, a.K = dy's channel stride,
//       a.Hin x a.Win = dy's size); a chunk lies in one plane and its 4 units are the plane's 2x2
//       taps at window (1 - py + a, 1 - px + b); the halo DMA gathers plane pixels (2ih + py,
//       2iw + px) -- the stride-2 4x4 conv of conv_fwd_v2 MODE 3 without its 12 zero taps.
// Weights (weight_prep_phase_kernel): unit u = chunk * 4 + q, [rows][32] per unit.
//
// PERS (persistent, one block per CU): the block walks the tiles v = blockIdx.x + k * gridDim.x
// (the tiles its XCD runs in the one-tile-per-block grid of ntiles blocks).  After a tile's
// epilogue staged its output in LDS and read it back into registers, the next tile's
// prologue DMA (weight stage 0, halo chunks 0 / 1) is issued and THEN the stores: every CU
// reaches its epilogue at the same time, so a tile's 128 KB of stores (HBM-bound as a burst)
// drain under the next tile's prologue instead of after it.
template <int WN, int WM, int RN, int RM, int NSB, int SCH = 0, int MODE = 0, bool PERS = false>
__global__ void __launch_bounds__(64 * WN * WM, (WN * RN * 16 >= 256 || WN == 1) ? 1 : 2)
conv3_halo_fwd3(ConvArgs a, unsigned x_bytes, int ntiles) {
  static_assert(MODE != 1 || (WN == 4 && RN == 4), "sub-pixel forward: one phase of 64 channels per wave column");
  constexpr int UPC = MODE ? 4 : 9;                        // tap units per 32-channel chunk
  constexpr int NW = WN * WM;
  constexpr int BN = WN * RN * 16, BM = WM * RM * 16, TR = BM / 64;
  static_assert(RM % 4 == 0, "a wave's pixels start on an image-row boundary of the tile");
  constexpr int PXB = 96;                                  // LDS bytes per halo pixel
  constexpr int HP = (TR + 2) * 66, HSL = HP * (PXB / 16), HQ = (HSL + 63) / 64, JH = (HQ + NW - 1) / NW;
  constexpr int HALO = HQ * 1024;
  // weight DMA pieces (16 rows) per tap: JB per wave, or one per wave for waves < QB when the
  // co tile has fewer pieces than waves (the 64-channel tile on 8 waves)
  constexpr int QB = BN / 16, JB = QB >= NW ? QB / NW : 1;
  static_assert(QB % NW == 0 || NW % QB == 0, "weight pieces per wave");
  constexpr int BST = BN * 64, STG = 2 * BST, WOFF = NSB * STG;
  constexpr int MAIN = WOFF + 2 * HALO, EPI = BM * BN * 2;
  static_assert(MAIN <= 163840, "LDS");
  static_assert(STG * (NSB - 1) + BST + (BN - 16) * 64 < 65536, "weight fragment immediates");
  __shared__ __attribute__((aligned(1024))) char smem[MAIN > EPI ? MAIN : EPI];

  FV_DIAG_BEGIN();
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int ntl = PERS ? ntiles : (int)gridDim.x;
  // tile of launch index v: the XCD-aware bijective remap (consecutive tiles on one XCD)
  auto remap = [&](int v) {
    const int q8 = ntl / 8, r8 = ntl % 8, x8 = v % 8;
    return (x8 < r8 ? x8 * (q8 + 1) : r8 * (q8 + 1) + (x8 - r8) * q8) + v / 8;
  };
  const int tiles_w = a.W >> 6, tiles_h = a.H / TR;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7fffffff, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);
  const int lrow = lane >> 2, lchk = lane & 3;
  // Weights are stage-major (weight_prep_body smaj): tap unit u = c * 9 + t is a [Cout][32]
  // block, so the 16 rows of a DMA piece are one contiguous KB (8 whole 128-B lines; the
  // [co][Kpad] rows made every piece 16 separate 64-B segments).  Piece jb of unit u starts at
  // u * ustep + (co0 + (wave + jb * NW) * 16) * 64; the lane's source chunk carries the LDS
  // chunk swizzle.
  const unsigned wstep = (unsigned)(NW * 16 * 64);
  const unsigned ustep = (unsigned)a.wus;
  const int nch = a.Cin >> 5, nsteps = UPC * nch / 2;
  const int cpp = a.Cin >> 7;                               // MODE 2: chunks per phase plane

  struct Tile {
    int tn, tm, tw, th, n, co0, p0;
    unsigned wbase;
  };
  auto tile_of = [&](int v) {
    Tile t;
    const int lid = remap(v);
    t.tn = lid % a.ntn;
    t.tm = lid / a.ntn;
    t.tw = t.tm % tiles_w;
    t.th = (t.tm / tiles_w) % tiles_h;
    t.n = t.tm / (tiles_w * tiles_h);
    t.co0 = t.tn * BN;
    t.p0 = (t.n * a.H + t.th * TR) * a.W + t.tw * 64;
    t.wbase = (unsigned)((t.co0 + wave * 16 + lrow) * 64 + ((lchk ^ rswz<bf16>(lrow)) << 4));
    return t;
  };
  // halo slots of this wave: slot k = 16-B chunk k % 6 of halo pixel k / 6 (chunks 4, 5 pad)
  unsigned hoff[JH];
  auto mk_hoff = [&](const Tile& t) {
#pragma unroll
    for (int j = 0; j < JH; ++j) {
      const int k = (wave + j * NW) * 64 + lane;
      const int hp = k / 6, ch = k - (k / 6) * 6;
      const int hr = hp / 66, hc = hp - (hp / 66) * 66;
      const int ih = t.th * TR + hr - 1, iw = t.tw * 64 + hc - 1;
      const bool ok = hp < HP && ch < 4 && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
      if constexpr (MODE == 2)     // plane (0, 0) pixel of dy; the chunk's plane is a uniform offset
        hoff[j] = ok ? (unsigned)((((t.n * a.Hin + 2 * ih) * a.Win + 2 * iw) * a.K + (ch << 3)) * 2) : 0x80000000u;
      else
        hoff[j] = ok ? (unsigned)(((((t.n * a.H + ih) * a.W + iw) << a.lgCin) + (ch << 3)) * 2) : 0x80000000u;
    }
  };
  auto issue_b = [&](unsigned wbase, int j, int buf) {
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int u = 2 * j + h;
      const unsigned Bs = sbase + buf * STG + h * BST;
#pragma unroll
      for (int jb = 0; jb < JB; ++jb)
        if (QB >= NW || wave < QB) dma16s(wr, Bs + (wave + jb * NW) * 1024, wbase, (unsigned)u * ustep + jb * wstep);
    }
  };
  // the step after whose barrier halo chunk c is issued: the last read of chunk c - 2 (same
  // buffer) was retired by it
  auto halo_step = [&](int c) { return MODE ? 2 * c - 3 : (9 * c - 10) / 2; };
  auto halo_soff = [&](int c) -> unsigned {
    if constexpr (MODE == 2) {
      const int pl = c / cpp, cc = c - pl * cpp;
      return (unsigned)((((pl >> 1) * a.Win + (pl & 1)) * a.K + cc * 32) * 2);
    } else {
      return (unsigned)(c * 64);
    }
  };
  auto issue_halo = [&](int c) {
    const unsigned Hs = sbase + WOFF + (c & 1) * HALO;
#pragma unroll
    for (int j = 0; j < JH; ++j)
      if (j < JH - 1 || wave + j * NW < HQ) dma16s(xr, Hs + (wave + j * NW) * 1024, hoff[j], halo_soff(c));
  };
  auto bcnt = [&](int j) { return j < nsteps && (QB >= NW || wave < QB) ? 2 * JB : 0; };
  // a tile's prologue DMA: weight stage 0, halo chunks 0 / 1, stages 1 .. NSB - 2
  auto issue_prologue = [&](const Tile& t) {
    issue_b(t.wbase, 0, 0);
    issue_halo(0);
    issue_halo(1);
    for (int i = 1; i < NSB - 1; ++i)
      if (i < nsteps) issue_b(t.wbase, i, i);
  };

  const int lr = lane & 15, lh = lane >> 4;
  // per-lane bases: weight row wn*RN*16 + lr (chunk swizzle is a function of lr only), halo
  // pixel of tile pixel wm*RM*16 + lr (RM*16 is a multiple of the 64-pixel tile row).  A tap
  // adds one wave-uniform offset to each (2 VALU per tap); the fragments are immediates.
  const int va = (wn * RN * 16 + lr) * 64 + ((lh ^ rswz<bf16>(lr)) << 4);
  const int vb = WOFF + ((wm * RM / 4) * 66 + lr) * PXB + lh * 16;
  auto load_frags = [&](Frag<bf16> (&fa)[RN], Frag<bf16> (&fb)[RM], int u, int buf) {
    int c, r, s3;
    if constexpr (MODE == 1) {
      c = u >> 2;
      r = (wn >> 1) + ((u >> 1) & 1);
      s3 = (wn & 1) + (u & 1);
    } else if constexpr (MODE == 2) {
      c = u >> 2;
      const int pl = c / cpp;
      r = ((u >> 1) & 1) + 1 - (pl >> 1);
      s3 = (u & 1) + 1 - (pl & 1);
    } else {
      c = u / 9;
      const int t = u - c * 9;
      r = t / 3;
      s3 = t - (t / 3) * 3;
    }
    const int pa = va + (buf * STG + (u & 1) * BST);
    const int pb = vb + ((c & 1) * HALO + (r * 66 + s3) * PXB);
#pragma unroll
    for (int i = 0; i < RN; ++i) fa[i].lds(smem + pa + i * 1024);
#pragma unroll
    for (int m = 0; m < RM; ++m) fb[m].lds(smem + pb + (((m * 16) >> 6) * 66 + ((m * 16) & 63)) * PXB);
  };
  const bool hi = wave >= NW / 2;                  // the second-dispatched wave of each SIMD
  const bool stag = (SCH & 2) && hi;

  int v = blockIdx.x;
  Tile t = tile_of(v);
  mk_hoff(t);
  issue_prologue(t);
  bool first = true;
  for (;;) {
    // the first reads need weight stage 0 and halo chunk 0 only: on the first tile the DMAs
    // issued after them (chunk 1, first read at unit UPC; stages 1 .. NSB - 2) stay in flight
    // past the prologue barrier and are waited for at the first step barriers; a later tile's
    // prologue was issued before the previous tile's stores, so all is waited for
    {
      const int nh1 = (JH - 1) + ((JH - 1) * NW + wave < HQ ? 1 : 0);
      int later = nh1;
      for (int i = 1; i < NSB - 1; ++i) later += bcnt(i);
      // a later tile: the previous epilogue's stores were issued after this prologue (vmcnt
      // retires in issue order on gfx9), so they may stay in flight too: NRES (+ 4 record
      // stores with store-pass records) per wave
      if (!first) later += BM * BN / (8 * NW * 64) + (MODE != 1 && a.spm ? 4 : 0);
      wait_vm_upto(later);
    }
    __syncthreads();
    FV_DIAG_PROLOGUE();
    f32x4 acc[RN][RM];
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[i][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    auto mfma_all = [&](const Frag<bf16> (&fa)[RN], const Frag<bf16> (&fb)[RM]) {
      if constexpr (!(SCH & 1)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
      for (int i = 0; i < RN; ++i)
#pragma unroll
        for (int m = 0; m < RM; ++m) acc[i][m] = mma(fa[i], fb[m], acc[i][m]);
      if constexpr (!(SCH & 1)) __builtin_amdgcn_s_setprio(0);
    };

    // the ring and halo schedule of conv3_halo_fwd2 (nch even: no odd last tap)
    Frag<bf16> fa0[RN], fb0[RM], fa1[RN], fb1[RM];
    int pend = 0;
    if (NSB - 1 < nsteps) {
      issue_b(t.wbase, NSB - 1, NSB - 1);
      pend = bcnt(NSB - 1);
    }
    load_frags(fa0, fb0, 0, 0);
    int hn = 2, hstep = halo_step(2);
    int bj = 0;
    if constexpr (SCH & 1) {
      if (hi) __builtin_amdgcn_s_setprio(1);
    }
    // barrier of step j: stage j + 1 landed (own DMAs counted, then the barrier publishes them),
    // and every wave's reads of stage j are done (its buffer is re-filled right after)
    auto step_barrier = [&]() {
      FV_DIAG_WAIT_BEGIN();
      if constexpr (NSB == 2) wait_vm<0>();
      else if (pend == 2 * JB) wait_vm<2 * JB>();
      else wait_vm_dyn(pend);
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      FV_DIAG_WAIT_END();
    };
    // stagger (SCH bit 1): waves NW/2.. take the barrier BEFORE the MFMAs of tap 2j (their
    // fragments are in registers), the others after; every read still falls in the same barrier
    // interval as in the lockstep order, so the ring / halo hazards are unchanged.
    // The last step is peeled: with it inside the loop (no barrier, no next-tap reads) the
    // wait-count pass merged its state into the loop's second MFMA cluster and made that
    // cluster wait for the next tap's fragment reads every step (lgkmcnt(7) .. (0)).
    for (int j = 0; j + 1 < nsteps; ++j) {
      load_frags(fa1, fb1, 2 * j + 1, bj);
      if constexpr ((SCH & 2) != 0) {
        if (stag) step_barrier();
      }
      mfma_all(fa0, fb0);
      const int bn1 = bj + 1 == NSB ? 0 : bj + 1;
      if (!stag) step_barrier();
      if (hn < nch && j == hstep) {
        issue_halo(hn);
        ++hn;
        hstep = halo_step(hn);
      }
      pend = 0;
      if (j + NSB < nsteps) {
        issue_b(t.wbase, j + NSB, bj);
        pend = bcnt(j + NSB);
      }
      load_frags(fa0, fb0, 2 * j + 2, bn1);
      FV_DIAG_ISSUE_END();
      mfma_all(fa1, fb1);
      bj = bn1;
    }
    load_frags(fa1, fb1, 2 * nsteps - 1, bj);
    mfma_all(fa0, fb0);
    mfma_all(fa1, fb1);
    if constexpr (SCH & 1) __builtin_amdgcn_s_setprio(0);
    FV_DIAG_LOOP_END();
    __syncthreads();
    const int vn = v + (int)gridDim.x;
    const bool nxt = PERS && vn < ntl;
    const Tile cur = t;
    if constexpr (PERS) {
      // the next tile's geometry and prologue DMA, issued between the epilogue's LDS read-back
      // and its stores (conv_epilogue / subpix_epilogue `mid`)
      auto mid = [&]() {
        if (nxt) {
          t = tile_of(vn);
          mk_hoff(t);
          issue_prologue(t);
        }
      };
      if constexpr (MODE == 1)
        subpix_epilogue<WM, RM>(a, acc, smem, cur.tn, cur.n, cur.th * TR, cur.tw * 64, cur.tm, wn, wm, lane, tid, mid);
      else
        conv_epilogue<bf16, WN, WM, RN, RM, true>(a, acc, smem, cur.co0, cur.p0, cur.tm, wn, wm, lane, tid, mid);
    } else {
      if constexpr (MODE == 1)
        subpix_epilogue<WM, RM>(a, acc, smem, cur.tn, cur.n, cur.th * TR, cur.tw * 64, cur.tm, wn, wm, lane, tid);
      else
        conv_epilogue<bf16, WN, WM, RN, RM, true>(a, acc, smem, cur.co0, cur.p0, cur.tm, wn, wm, lane, tid);
    }
    FV_DIAG_END();
    if (!nxt) break;
    v = vn;
    first = false;
  }
}

// ----------------------------------------------------------------------------------------
// Halo-tiled 7x7 forward for a small channel side (bf16): AFE.in_conv 3->64 forward,
// Generator.out_conv 64->3 forward and its 3->64 backward-data.  The block's TR x 64 output
// pixels plus the (KS-1)-pixel halo of the input are staged in LDS ONCE (DMA, per-lane
// source addressing, zero border from the buffer range check); every tap then reads its
// shifted window from LDS, instead of the 49x im2col re-read of the generic path.
//   A fragment (16 pixels x 32 k): lane (i, g) reads the 16-B chunk g of k-step ks at halo
//   pixel (pixel i + tap offset) -> one ds_read_b128; 16-B chunks inside a pixel are XOR-
//   swizzled by the pixel index (conflict-light reads of 128-B pixels).
//   B fragment (weights [co][Kpad]): from LDS with padded rows (WLDS) or straight from
//   global/L1 (3 output channels: 16 padded rows, 100 KB, cache-resident).
// 8 waves; wave w owns pixels [w*RM*16, (w+1)*RM*16) of the tile and all RN*16 channels.
// Requires W % 64 == 0 and H % TR == 0 (host checks).
// ----------------------------------------------------------------------------------------
template <int KS, int CIN, int RN, int TR, bool WLDS, bool KSPLIT>
__global__ void __launch_bounds__(512, 4)
conv_halo_fwd(ConvArgs a, unsigned x_bytes) {
  constexpr int PAD = KS / 2, TW = 64;
  constexpr int MT = TR * 4;                       // 16-pixel m-tiles per block
  // KSPLIT: every wave owns all MT m-tiles and 1/8 of the k-steps (partials summed in LDS);
  // otherwise wave w owns m-tiles [w*RM, (w+1)*RM) and all k-steps.
  constexpr int RM = KSPLIT ? MT : MT / 8;
  constexpr int HR = TR + KS - 1, HW = TW + KS - 1;
  constexpr int CPP = CIN / 8;                     // 16-B chunks per pixel
  constexpr int HCH = HR * HW * CPP;               // halo chunks
  constexpr int HQ = (HCH + 63) / 64;              // 1-KB pieces
  constexpr int KPAD = ((KS * KS * CIN + 31) / 32) * 32;
  constexpr int NKS = KPAD / 32;
  constexpr int KPW = (NKS + 7) / 8;               // k-steps per wave (KSPLIT)
  constexpr int WROW = KPAD / 8 + 1;               // padded weight row (16-B chunks)
  constexpr int WCH = RN * 16 * WROW;
  constexpr int WQ = WLDS ? (WCH + 63) / 64 : 0;
  constexpr int HB = HQ * 1024, WB = WQ * 1024;
  constexpr int SCR = 4096;                        // epilogue scratch (BN partials)
  static_assert(!KSPLIT || (RN == 1 && !WLDS && 8 * MT * 1024 <= HB), "k-split layout");
  __shared__ __attribute__((aligned(1024))) char smem[HB + WB + SCR];
  char* halo = smem;
  char* wlds = smem + HB;

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_w = a.W / TW, tiles_h = a.H / TR;
  const int tile = blockIdx.x;
  const int n = tile / (tiles_h * tiles_w);
  const int rem = tile - n * tiles_h * tiles_w;
  const int h0 = (rem / tiles_w) * TR, w0 = (rem % tiles_w) * TW;
  const int li = lane & 15, g = lane >> 4;
  const bf16* __restrict__ wk = reinterpret_cast<const bf16*>(a.w);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  for (int q = wave; q < HQ; q += 8) {
    const int L = q * 64 + lane;
    const int hp = L / CPP, ch = L - (L / CPP) * CPP;
    const int hr = hp / HW, hc = hp - (hp / HW) * HW;
    const int hh = h0 + hr - PAD, ww = w0 + hc - PAD;
    const int sc = ch ^ (hp & (CPP - 1));
    const bool ok = L < HCH && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
    const unsigned off = ok ? (unsigned)((((n * a.H + hh) * a.W + ww) * CIN + sc * 8) * 2) : 0x80000000u;
    dma16(xr, halo + q * 1024, off);
  }
  if constexpr (WLDS) {
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7fffffff, 0x00020000);
    for (int q = wave; q < WQ; q += 8) {
      const int L = q * 64 + lane;
      const int row = L / WROW, ch = L - (L / WROW) * WROW;
      const bool ok = L < WCH && ch < KPAD / 8;
      const unsigned off = ok ? (unsigned)((row * a.Kpad + ch * 8) * 2) : 0x80000000u;
      dma16(wr, wlds + q * 1024, off);
    }
  }
  const int ks0 = KSPLIT ? wave * KPW : 0;
  const int ks1 = KSPLIT ? min(NKS, ks0 + KPW) : NKS;
  bf16x8 bpre[KSPLIT ? KPW : 1];
  if constexpr (KSPLIT) {   // this wave's weight fragments, straight to registers
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      const int kc = (ks0 + j) * 4 + g;
      bpre[j] = (ks0 + j < NKS) ? *reinterpret_cast<const bf16x8*>(wk + (long)li * a.Kpad + kc * 8) : bf16x8{};
    }
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  f32x4 acc[RN][RM];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int j = 0; j < RM; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  int hbase[RM];   // halo pixel of this lane's output pixel, per m-tile (tap (0,0))
#pragma unroll
  for (int m = 0; m < RM; ++m) {
    const int loc = (KSPLIT ? 0 : wave * RM * 16) + m * 16 + li;
    hbase[m] = (loc / TW) * HW + (loc % TW);
  }
  auto kstep = [&](int ks, const bf16x8 (&bfr)[RN]) {
    const int kc = ks * 4 + g;                 // this lane's 16-B k chunk
    const int tap = kc / CPP, ch = kc - (kc / CPP) * CPP;
    const bool kin = tap < KS * KS;
    const int r = tap / KS, s = tap - (tap / KS) * KS;
    const int toff = r * HW + s;
    bf16x8 afr[RM];
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int hp = hbase[m] + toff;
      bf16x8 v = *reinterpret_cast<const bf16x8*>(halo + (hp * CPP + (ch ^ (hp & (CPP - 1)))) * 16);
      if (!kin) v = bf16x8{};
      afr[m] = v;
    }
#pragma unroll
    for (int nn = 0; nn < RN; ++nn)
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[nn][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nn], afr[m], acc[nn][m], 0, 0, 0);
  };
  if constexpr (KSPLIT) {
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
      if (ks0 + j < ks1) {
        const bf16x8 bfr[RN] = {bpre[j]};
        kstep(ks0 + j, bfr);
      }
    }
  } else {
#pragma unroll 2
    for (int ks = ks0; ks < ks1; ++ks) {
      const int kc = ks * 4 + g;
      bf16x8 bfr[RN];
#pragma unroll
      for (int nn = 0; nn < RN; ++nn) {
        if constexpr (WLDS) bfr[nn] = *reinterpret_cast<const bf16x8*>(wlds + ((nn * 16 + li) * WROW + kc) * 16);
        else bfr[nn] = *reinterpret_cast<const bf16x8*>(wk + (long)(nn * 16 + li) * a.Kpad + kc * 8);
      }
      kstep(ks, bfr);
    }
  }
  const int p0 = (n * a.H + h0) * a.W + w0;
  if constexpr (KSPLIT) {
    // sum the 8 waves' partial tiles through LDS (halo no longer needed); wave w finishes m-tile w
    __syncthreads();
    f32x4* red = reinterpret_cast<f32x4*>(halo);
#pragma unroll
    for (int m = 0; m < RM; ++m) red[(wave * RM + m) * 64 + lane] = acc[0][m];
    __syncthreads();
    f32x4 t[1][1];
    t[0][0] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int w = 0; w < 8; ++w) t[0][0] += red[(w * RM + wave) * 64 + lane];
    conv_epilogue<bf16, 1, 8, 1, 1>(a, t, smem + HB + WB, 0, p0, tile, 0, wave, lane, tid);
  } else {
    conv_epilogue<bf16, 1, 8, RN, RM>(a, acc, smem + HB + WB, 0, p0, tile, 0, wave, lane, tid);
  }
}

// ----------------------------------------------------------------------------------------
// conv7c4_fwd: 7x7, <= 4 valid input channels (stored as 8) -> 64 output channels:
// AFE.in_conv 3 -> 64 forward (models.py:932) and Generator.out_conv's data gradient (3 -> 64).
// conv_halo_fwd<7, 8, ...> pads K to 49 taps x 8 channels = 416 (62 % zeros) and restages the
// 54 KB weight image in every one of its 8192 blocks (the LDS-DMA of the weights, not the
// MFMAs, set its 153-191 us).  Here:
//  * K packs 2 taps x 4 channels per 16-B fragment chunk: k = r * 32 + s * 4 + ci (s = 7 and
//    ci >= cin_valid are zero weights), K = 7 x 32 = 224 -> 7 MFMA k-steps instead of 13; the
//    A fragment of lane (pixel i, chunk g) is halo pixels (i + 2g, i + 2g + 1) of row r, 8 B
//    each (two ds_read_b64 from the 16-B NHWC pixels);
//  * persistent blocks (2 per CU): the 64 x 224 weight image is staged ONCE per block, the
//    halos of the next two tiles are in flight (3-buffer ring) while the current one computes;
//  * a minimal epilogue (bias preloaded, NHWC bf16 stores widened to 16 B), so no load in the
//    loop waits behind the halo DMA; ONE BN (sum, sum^2) record per BLOCK (r6): every lane
//    keeps the running sums of its 16 channels over all the block's tiles (plain adds), reduced
//    across lanes and waves once at the end -- the per-tile record (32 DPP row sums per wave
//    and tile, an LDS exchange and a record store) made the in_conv forward 27 us slower than
//    the same kernel without statistics (104 vs 77 us in the replayed step).  Block b owns tiles
//    b, b + G, ... (C74 tiles per block, c74_grid), so record b covers exactly those pixels.
// Tile: 4 rows x 64 columns x 64 co; wave w owns pixels [32w, 32w + 32) x all 64 co.
// ----------------------------------------------------------------------------------------
constexpr int C74_TR = 4, C74_HW = 71, C74_HR = C74_TR + 6;          // halo row: 64 + 6 + 1 (zero) px
constexpr int C74_K = 224, C74_WCOL = C74_K / 8;                     // 16-B chunks (k columns) per weight row
constexpr int C74_WQ = 64 * C74_WCOL / 64;                           // 1-KB weight pieces (28)
constexpr int C74_HQ = (C74_HR * C74_HW + 63) / 64;                  // 1-KB halo pieces (16 B / px)
__global__ void __launch_bounds__(512, 2)
conv7c4_fwd(ConvArgs a, unsigned x_bytes, int ntiles) {
  constexpr int WB = C74_WQ * 1024, HB = C74_HQ * 1024, NHB = 3;   // 3-deep halo ring
  __shared__ __attribute__((aligned(1024))) char smem[WB + NHB * HB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int tiles_w = a.W >> 6, tiles_h = a.H / C74_TR;
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7fffffff, 0x00020000);

  // halo pieces of this wave (pixel L = q * 64 + lane of the 10 x 71 halo, 16 B each)
  auto issue_halo = [&](int tile, int buf) {
    const int n = tile / (tiles_h * tiles_w), rem = tile - n * tiles_h * tiles_w;
    const int h0 = (rem / tiles_w) * C74_TR, w0 = (rem % tiles_w) * 64;
    for (int q = wave; q < C74_HQ; q += 8) {
      const int L = q * 64 + lane;
      const int hr = L / C74_HW, hc = L - (L / C74_HW) * C74_HW;
      const int hh = h0 + hr - 3, ww = w0 + hc - 3;
      const bool ok = L < C74_HR * C74_HW && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      dma16s(xr, sbase + WB + buf * HB + q * 1024, ok ? (unsigned)((((n * a.H + hh) * a.W + ww) * 8) * 2) : 0x80000000u, 0u);
    }
  };
  // weight image [n-tile][k column][16 rows] of 16-B chunks: the 16 lanes of every ds_read_b128
  // lane group read 16 different rows of one column = 16 different bank slots (the padded
  // [row][29] image put 2 lanes of a group on one slot: 50 % of the LDS cycles were bank
  // conflicts, profiles/r6/r6_convpmc_7x7.txt)
  for (int q = wave; q < C74_WQ; q += 8) {
    const int L = q * 64 + lane;
    const int li = L & 15, t = L >> 4, col = t % C74_WCOL, row = (t / C74_WCOL) * 16 + li;
    dma16s(wr, sbase + q * 1024, (unsigned)((row * C74_K + col * 8) * 2), 0u);
  }
  int tile = blockIdx.x;
  if (tile < ntiles) issue_halo(tile, 0);
  if (tile + (int)gridDim.x < ntiles) issue_halo(tile + gridDim.x, 1);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();

  float bv[4][4];
#pragma unroll
  for (int nn = 0; nn < 4; ++nn)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[nn][i] = a.bias ? a.bias[nn * 16 + g * 4 + i] : 0.f;
  // halo pixel of this lane's output pixel (tap (0, 0)) per m-tile; the tile is 4 rows x 64
  int hbase[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int loc = wave * 32 + m * 16 + li;
    hbase[m] = (loc >> 6) * C74_HW + (loc & 63);
  }
  // BN running sums of this lane's channels nn * 16 + g * 4 + i over the block's pixels
  float bs[4][4], bq[4][4];
#pragma unroll
  for (int nn = 0; nn < 4; ++nn)
#pragma unroll
    for (int i = 0; i < 4; ++i) bs[nn][i] = bq[nn][i] = 0.f;
  int buf = 0;
  for (; tile < ntiles; tile += gridDim.x) {
    // the halo two tiles ahead goes into the buffer the previous tile released at its barrier
    const int ahead = tile + 2 * gridDim.x;
    if (ahead < ntiles) issue_halo(ahead, buf == 0 ? 2 : buf - 1);
    f32x4 acc[4][2];
#pragma unroll
    for (int nn = 0; nn < 4; ++nn)
#pragma unroll
      for (int m = 0; m < 2; ++m) acc[nn][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* hs = smem + WB + buf * HB;
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      bf16x8 bfr[4], afr[2];
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
        bfr[nn] = *reinterpret_cast<const bf16x8*>(smem + ((nn * C74_WCOL + r * 4 + g) * 16 + li) * 16);
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        const char* p = hs + (hbase[m] + r * C74_HW + 2 * g) * 16;
        const uint2 lo = *reinterpret_cast<const uint2*>(p), hi = *reinterpret_cast<const uint2*>(p + 16);
        afr[m] = __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
      }
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
#pragma unroll
        for (int m = 0; m < 2; ++m) acc[nn][m] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(bfr[nn], afr[m], acc[nn][m], 0, 0, 0);
    }
    // epilogue: bias, BN records (one per 32-pixel wave row, as conv_epilogue), NHWC stores
    const int n = tile / (tiles_h * tiles_w), rem = tile - n * tiles_h * tiles_w;
    const int p0 = (n * a.H + (rem / tiles_w) * C74_TR) * a.W + (rem % tiles_w) * 64;
#pragma unroll
    for (int nn = 0; nn < 4; ++nn)
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int i = 0; i < 4; ++i) acc[nn][m][i] += bv[nn][i];
    if (a.stats) {
#pragma unroll
      for (int nn = 0; nn < 4; ++nn)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          const float v0 = acc[nn][0][i], v1 = acc[nn][1][i];
          bs[nn][i] += v0 + v1;
          bq[nn][i] += v0 * v0 + v1 * v1;
        }
    }
    // 16-B stores (the guide's T21 widening, 16-lane rows): lane (li, g) holds channels
    // nt * 16 + g * 4 .. + 3 of every n-tile nt; one v_permlane16_swap per dword of an n-tile
    // pair (2q, 2q + 1) leaves lane g with the 8 contiguous channels (2q + (g & 1)) * 16 +
    // (g >> 1) * 8 .. + 7: 4 dwordx4 stores per lane and tile instead of 8 dwordx2
    auto pk = [](float lo, float hi) {
      const bf16 t[2] = {(bf16)lo, (bf16)hi};
      return *reinterpret_cast<const unsigned*>(t);
    };
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int loc = wave * 32 + m * 16 + li;
      bf16* yp = reinterpret_cast<bf16*>(a.y) + (long)(p0 + (loc >> 6) * a.W + (loc & 63)) * a.ldy;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 va = acc[2 * q][m], vb = acc[2 * q + 1][m];
        const auto s0 = __builtin_amdgcn_permlane16_swap(pk(va[0], va[1]), pk(vb[0], vb[1]), false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pk(va[2], va[3]), pk(vb[2], vb[3]), false, false);
        *reinterpret_cast<uint4*>(yp + (2 * q + (g & 1)) * 16 + (g >> 1) * 8) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    }
    // the next tile's halo was issued a whole tile earlier; younger than it are exactly the
    // previous tile's 4 stores, this tile's BN record store (waves 0-1), its halo DMA pieces
    // (2 / 1 per wave, when the tile two ahead exists) and its 4 stores: waiting for that count
    // leaves all of them in flight (vmcnt(8) made every tile wait for half of the previous
    // tile's stores); the barrier publishes it to all waves and releases this tile's buffer
    // (raw barrier: __syncthreads() would also drain the stores)
    {
      const int dpieces = ahead < ntiles ? (wave + 8 < C74_HQ ? 2 : 1) : 0;
      wait_vm_dyn(8 + dpieces);
    }
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    buf = buf == 2 ? 0 : buf + 1;
  }
  if (a.stats) {
    // the block's record: lane sums over li (row16_sum), then the 8 waves in order through LDS
    // (the halo ring is free: every wave passed the last tile's barrier)
    float* sw = reinterpret_cast<float*>(smem + WB);
#pragma unroll
    for (int nn = 0; nn < 4; ++nn)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        const float sv = row16_sum(bs[nn][i]), qv = row16_sum(bq[nn][i]);
        if (li == 0) {
          sw[wave * 128 + nn * 16 + g * 4 + i] = sv;
          sw[wave * 128 + 64 + nn * 16 + g * 4 + i] = qv;
        }
      }
    __syncthreads();
    if (tid < 128 && (int)blockIdx.x < a.nrec) {
      float v = 0.f;
#pragma unroll
      for (int w = 0; w < 8; ++w) v += sw[w * 128 + tid];
      a.stats[(long)blockIdx.x * 128 + tid] = v;
    }
  }
}

// ----------------------------------------------------------------------------------------
// 3x3 conv with 64 input channels at full resolution (AFE.down1 forward, 64 -> 128 at 256^2),
// as a sliding band with the weights in registers.  A block of 8 waves owns 64 output channels
// of one 64-column strip of one image and walks a band of rows, 4 output rows per iteration:
// wave (rw, cg) computes output row h0 + rw x 64 pixels for the 32 channels cg of the block's
// 64, with its 2 x 18 A fragments (32 co x K = 576 = 9 taps x 64 ci) held in registers for the
// whole band (two waves per SIMD fit: ~240 registers each) -- the only LDS traffic is the input,
// 4 B fragments per 8 MFMAs.  Input rows (66 px incl. the halo columns) stream through a 10-row
// LDS ring by LDS-DMA (44 pieces per iteration spread over the waves and over the first k-steps)
// and are waited for one iteration later (counted vmcnt: the output stores issued after them
// stay in flight).  A halo pixel takes 160 B (128 B of channels + 32 B zero-filled by
// out-of-range DMA slots): 16 consecutive pixels read by ds_read_b128 are conflict-free from any
// start.  The two 64-channel halves of a strip are neighbours on one XCD, so the input is
// fetched from HBM about once.  Epilogue per iteration: bias, BN (sum, sum of squares) per lane
// over 8 iterations = one record of 512 pixels per (wave row, 8 iterations), 16-B bf16 stores
// (v_permlane16_swap pairs the two 16-channel fragments).  Replaces conv_fwd_v2's per-tap DMA.
// ----------------------------------------------------------------------------------------
constexpr int C64_PXB = 160, C64_ROWB = 11 * 1024, C64_NR = 10, C64_G = 8;
__global__ void __launch_bounds__(512, 1)
conv3c64_fwd(ConvArgs a, unsigned x_bytes, int nbands) {
  __shared__ __attribute__((aligned(1024))) char smem[C64_NR * C64_ROWB];
  __shared__ __attribute__((aligned(16))) float sbias[64];              // the block's 64 biases
  // per-lane BN partial sums of the current 8-iteration record group, [wave][16][lane] (kept
  // in LDS: their 16 registers double-buffer the B fragments instead)
  __shared__ __attribute__((aligned(16))) float sacc[8 * 16 * 64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wave & 1, rw = wave >> 1;
  const int lr = lane & 15, lh = lane >> 4;
  // XCD-aware order: consecutive local ids (the co groups of one strip) share an XCD
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int nco = a.Cout >> 6, strips = a.W >> 6;
  const int cgrp = lid % nco, rest = lid / nco;
  const int band = rest % nbands, strip = (rest / nbands) % strips, n = rest / (nbands * strips);
  const int BAND = a.H / nbands, hb = band * BAND, w0 = strip * 64;
  const int cw = cgrp * 64 + cg * 32;                       // this wave's first output channel

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);
  // DMA slots of a row: 16-B chunk k = piece * 64 + lane -> halo pixel k / 10, chunk k % 10
  // (recomputed per piece: a register table of the 11 offsets does not fit beside the weights)
  auto poff_of = [&](int p, int ln) {
    const int k = p * 64 + ln, px = k / 10, ch = k - px * 10;
    const int iw = w0 - 1 + px;
    return (px < 66 && ch < 8 && iw >= 0 && iw < a.W) ? (unsigned)((iw * 64 + ch * 8) * 2) : 0x80000000u;
  };
  auto row_slot = [&](int y) { return (y - hb + 1) % C64_NR; };
  // piece q (0 .. 11 * rows - 1) of the rows starting at y0: row y0 + q / 11, piece q % 11
  auto issue_piece = [&](int y0, int q) {                  // rows outside the image -> zeros
    const int y = y0 + q / 11, p = q % 11;
    const bool rok = y >= 0 && y < a.H;
    const unsigned v = poff_of(p, lane);
    dma16s(xr, sbase + row_slot(y) * C64_ROWB + p * 1024, rok ? v : 0x80000000u,
           rok ? (unsigned)((n * a.H + y) * a.W) * 128u : 0u);
  };

  // the wave's weights: A fragment (cf, ks) = 16 channels x 32 k, k = tap * 64 + ci
  bf16x8 wf[2][18];
  const bf16* wk = reinterpret_cast<const bf16*>(a.w);
#pragma unroll
  for (int cf = 0; cf < 2; ++cf)
#pragma unroll
    for (int ks = 0; ks < 18; ++ks)
      wf[cf][ks] = *reinterpret_cast<const bf16x8*>(wk + (long)(cw + cf * 16 + lr) * a.Kpad + ks * 32 + lh * 8);

  // prologue: input rows hb - 1 .. hb + 4 (66 pieces)
  for (int q = wave; q < 66; q += 8) issue_piece(hb - 1, q);
  // biases in LDS, read back per epilogue: 8 registers fewer beside the 144 weight registers
  // (loaded after the prologue DMA is on its way)
  if (tid < 64) sbias[tid] = a.bias ? a.bias[cgrp * 64 + tid] : 0.f;
  __syncthreads();

  float* const sa = sacc + wave * 16 * 64 + lane;         // element e at sa[e * 64]
  const int niter = BAND >> 2, ng = niter / C64_G;
  const int rec0 = ((n * strips + strip) * nbands + band) * (4 * ng);
  const int loff = lr * C64_PXB + lh * 16;
  auto pk = [](float lo, float hi) {
    const bf16 t[2] = {(bf16)lo, (bf16)hi};
    return *reinterpret_cast<const unsigned*>(t);
  };

  for (int it = 0; it < niter; ++it) {
    const int h0 = hb + 4 * it;
    // this iteration's rows landed; younger than them are at most the previous iteration's 4
    // output stores (+ 2 record stores), which stay in flight
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = it + 1 < niter;
    const int orow = h0 + rw;
    unsigned sb[3];
#pragma unroll
    for (int q = 0; q < 3; ++q) sb[q] = (unsigned)(row_slot(orow - 1 + q) * C64_ROWB + loff);

    f32x4 acc[4][2];
#pragma unroll
    for (int pf = 0; pf < 4; ++pf)
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) acc[pf][cf] = f32x4{0.f, 0.f, 0.f, 0.f};
    // B fragments double-buffered: k-step ks + 1's are read before k-step ks's MFMAs
    auto ldb = [&](bf16x8 (&fb)[4], int ks) {
      const int tap = ks >> 1, r = tap / 3, s = tap - (tap / 3) * 3, ch = ks & 1;
#pragma unroll
      for (int pf = 0; pf < 4; ++pf)
        fb[pf] = *reinterpret_cast<const bf16x8*>(smem + sb[r] + (pf * 16 + s) * C64_PXB + ch * 64);
    };
    bf16x8 fbq[2][4];
    ldb(fbq[0], 0);
#pragma unroll
    for (int ks = 0; ks < 18; ++ks) {
      if (ks + 1 < 18) ldb(fbq[(ks + 1) & 1], ks + 1);
      const bf16x8 (&fb)[4] = fbq[ks & 1];
      // the next iteration's rows h0 + 5 .. h0 + 8: pieces wave, wave + 8, ... < 44
      if (ks < 6 && more && wave + 8 * ks < 44) issue_piece(h0 + 5, wave + 8 * ks);
#pragma unroll
      for (int pf = 0; pf < 4; ++pf)
#pragma unroll
        for (int cf = 0; cf < 2; ++cf)
          acc[pf][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cf][ks], fb[pf], acc[pf][cf], 0, 0, 0);
    }

    // epilogue: bias, BN partials, 16-B stores: lane (lr, lh) holds channels cf * 16 + lh * 4
    // .. + 3 of pixel lr; one v_permlane16_swap per dword pair leaves lane lh with the 8
    // contiguous channels (lh & 1) * 16 + (lh >> 1) * 8 .. + 7
    bf16* yp = reinterpret_cast<bf16*>(a.y) + ((long)(n * a.H + orow) * a.W + w0 + lr) * a.ldy + cw +
               (lh & 1) * 16 + (lh >> 1) * 8;
    float st[2][4], sq[2][4];
    const bool g0 = (it % C64_G) == 0;                    // the record group's first iteration
#pragma unroll
    for (int cf = 0; cf < 2; ++cf)
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        st[cf][i] = g0 ? 0.f : sa[(cf * 4 + i) * 64];
        sq[cf][i] = g0 ? 0.f : sa[(8 + cf * 4 + i) * 64];
      }
#pragma unroll
    for (int pf = 0; pf < 4; ++pf) {
      float v[2][4];
#pragma unroll
      for (int cf = 0; cf < 2; ++cf)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          v[cf][i] = acc[pf][cf][i] + sbias[cg * 32 + cf * 16 + lh * 4 + i];
          st[cf][i] += v[cf][i];
          sq[cf][i] += v[cf][i] * v[cf][i];
        }
      const auto s0 = __builtin_amdgcn_permlane16_swap(pk(v[0][0], v[0][1]), pk(v[1][0], v[1][1]), false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(pk(v[0][2], v[0][3]), pk(v[1][2], v[1][3]), false, false);
      *reinterpret_cast<uint4*>(yp + (long)pf * 16 * a.ldy) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
    if ((it % C64_G) != C64_G - 1) {
#pragma unroll
      for (int cf = 0; cf < 2; ++cf)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sa[(cf * 4 + i) * 64] = st[cf][i];
          sa[(8 + cf * 4 + i) * 64] = sq[cf][i];
        }
    } else if (a.stats) {
      // record (block, 8-iteration group, wave row): lanes 0-3 of a 16-lane row store the 4
      // channel sums, lanes 4-7 the squares (conv_epilogue's record layout)
      const int rec = rec0 + (it / C64_G) * 4 + rw;
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) {
        float sv[4], qv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sv[i] = row16_sum(st[cf][i]);
          qv[i] = row16_sum(sq[cf][i]);
        }
        const int cb = cw + cf * 16 + lh * 4, ii = lr & 3;
        const float s01 = ii & 1 ? sv[1] : sv[0], s23 = ii & 1 ? sv[3] : sv[2];
        const float q01 = ii & 1 ? qv[1] : qv[0], q23 = ii & 1 ? qv[3] : qv[2];
        const float val = lr < 4 ? (ii & 2 ? s23 : s01) : (ii & 2 ? q23 : q01);
        if (lr < 8 && rec < a.nrec) a.stats[(long)(rec * 2 + (lr >> 2)) * a.Cout + cb + ii] = val;
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// conv3up_band_fwd: the UpBlock2D forward (nearest x2 upsample + 3x3 as 4 sub-pixel phases of a
// 2x2 conv over the low-res input, modules.py:78-89) for a 128-channel input, as a sliding band
// like conv3c64_fwd: a block owns (image, 32-column low-res strip = 64 output columns, 64 output
// channels, band of low-res rows); wave (phase pa pb, 32-channel group cg) keeps its phase's
// 32 co x K = 4 taps x 128 ci weights as MFMA A fragments in registers (128 VGPRs) for the whole
// band, so the only LDS traffic is the input: low-res rows (34 pixels incl. the column halo) land
// ONCE by LDS-DMA in a 6-row ring (272-B pixels: 16 consecutive pixels read by ds_read_b128 are
// conflict-free) -- the halo kernel (MODE 1) restaged a 4-row halo per 32-channel chunk for only
// 4 taps of work, bandwidth-bound.  An iteration = 2 low-res rows (4 output rows); wave (pa, pb)
// writes output rows 2h + pa, columns 2w + pb.  Epilogue: bias, BN records of 256 pixels
// (4 iterations x 2 rows x 32 columns of one phase; the two channel-group waves of the phase fill
// the record's 64 channels), 16-B stores (v_permlane16_swap pairs the 16-channel fragments).
// Weights: the sub-pixel layout of weight_prep_subpix_kernel, wk [4][rows][Kpad = 512].
// ----------------------------------------------------------------------------------------
constexpr int UPB_PXB = 272, UPB_ROWB = 10 * 1024, UPB_NR = 6, UPB_G = 4;
__global__ void __launch_bounds__(512, 1)
conv3up_band_fwd(ConvArgs a, unsigned x_bytes, int nbands) {
  __shared__ __attribute__((aligned(1024))) char smem[UPB_NR * UPB_ROWB];
  __shared__ __attribute__((aligned(16))) float sbias[64];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int cg = wave & 1, ph = wave >> 1, pa = ph >> 1, pb = ph & 1;
  const int lr = lane & 15, lh = lane >> 4;
  // XCD-aware order: consecutive local ids (the co groups of one strip) share an XCD
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int nco = a.Cout >> 6, strips = a.Win >> 5;
  const int cgrp = lid % nco, rest = lid / nco;
  const int band = rest % nbands, strip = (rest / nbands) % strips, n = rest / (nbands * strips);
  const int BAND = a.Hin / nbands, hb = band * BAND, wl0 = strip * 32;
  const int cw = cgrp * 64 + cg * 32;                        // this wave's first output channel

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);
  // DMA slots of a row: 16-B chunk k = piece * 64 + lane -> LDS pixel k / 17 (low-res column
  // wl0 - 1 + k / 17), chunk k % 17 (chunk 16: the pad)
  auto poff_of = [&](int p, int ln) {
    const int k = p * 64 + ln, px = k / 17, ch = k - px * 17;
    const int iw = wl0 - 1 + px;
    return (px < 34 && ch < 16 && iw >= 0 && iw < a.Win) ? (unsigned)((iw * 128 + ch * 8) * 2) : 0x80000000u;
  };
  auto row_slot = [&](int y) { return (y - hb + 1) % UPB_NR; };
  // piece q (0 .. 10 * rows - 1) of the rows starting at y0: row y0 + q / 10, piece q % 10
  auto issue_piece = [&](int y0, int q) {                  // rows outside the image -> zeros
    const int y = y0 + q / 10, p = q % 10;
    const bool rok = y >= 0 && y < a.Hin;
    dma16s(xr, sbase + row_slot(y) * UPB_ROWB + p * 1024, rok ? poff_of(p, lane) : 0x80000000u,
           rok ? (unsigned)((n * a.Hin + y) * a.Win) * 256u : 0u);
  };

  // the wave's weights: A fragment (cf, ks) = 16 channels x 32 k, k = (rr * 2 + ss) * 128 + ci
  bf16x8 wf[2][16];
  const bf16* wk = reinterpret_cast<const bf16*>(a.w) + (long)ph * a.wphase;
#pragma unroll
  for (int cf = 0; cf < 2; ++cf)
#pragma unroll
    for (int ks = 0; ks < 16; ++ks)
      wf[cf][ks] = *reinterpret_cast<const bf16x8*>(wk + (long)(cw + cf * 16 + lr) * a.Kpad + ks * 32 + lh * 8);

  // prologue: low-res rows hb - 1 .. hb + 2 (40 pieces)
  for (int q = wave; q < 40; q += 8) issue_piece(hb - 1, q);
  if (tid < 64) sbias[tid] = a.bias ? a.bias[cgrp * 64 + tid] : 0.f;
  __syncthreads();

  float st[2][4], sq[2][4];
#pragma unroll
  for (int cf = 0; cf < 2; ++cf)
#pragma unroll
    for (int i = 0; i < 4; ++i) st[cf][i] = sq[cf][i] = 0.f;
  const int niter = BAND >> 1, ng = niter / UPB_G;
  const int rec0 = ((n * strips + strip) * nbands + band) * (4 * ng);
  auto pk = [](float lo, float hi) {
    const bf16 t[2] = {(bf16)lo, (bf16)hi};
    return *reinterpret_cast<const unsigned*>(t);
  };

  for (int it = 0; it < niter; ++it) {
    const int h0 = hb + 2 * it;
    // this iteration's rows landed; younger than them are at most the previous iteration's 4
    // output stores (+ record stores), which stay in flight
    if (it == 0) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const bool more = it + 1 < niter;
#pragma unroll
    for (int hh = 0; hh < 2; ++hh) {
      const int h = h0 + hh;
      // input rows h + pa - 1 + rr, LDS pixel of output column w: w + pb + ss (halo offset 1)
      unsigned sb[2];
#pragma unroll
      for (int rr = 0; rr < 2; ++rr) sb[rr] = (unsigned)(row_slot(h + pa - 1 + rr) * UPB_ROWB + (lr + pb) * UPB_PXB + lh * 16);
      auto ldb = [&](bf16x8 (&fb)[2], int ks) {
        const int tap = ks >> 2, rr = tap >> 1, ss = tap & 1, cc = ks & 3;
#pragma unroll
        for (int m = 0; m < 2; ++m)
          fb[m] = *reinterpret_cast<const bf16x8*>(smem + sb[rr] + (m * 16 + ss) * UPB_PXB + cc * 64);
      };
      f32x4 acc[2][2];
#pragma unroll
      for (int m = 0; m < 2; ++m)
#pragma unroll
        for (int cf = 0; cf < 2; ++cf) acc[m][cf] = f32x4{0.f, 0.f, 0.f, 0.f};
      bf16x8 fbq[2][2];
      ldb(fbq[0], 0);
#pragma unroll
      for (int ks = 0; ks < 16; ++ks) {
        if (ks + 1 < 16) ldb(fbq[(ks + 1) & 1], ks + 1);
        // the next iteration's rows h0 + 3, h0 + 4: pieces wave, wave + 8, wave + 16 < 20
        if (hh == 0 && ks < 3 && more && wave + 8 * ks < 20) issue_piece(h0 + 3, wave + 8 * ks);
#pragma unroll
        for (int m = 0; m < 2; ++m)
#pragma unroll
          for (int cf = 0; cf < 2; ++cf)
            acc[m][cf] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[cf][ks], fbq[ks & 1][m], acc[m][cf], 0, 0, 0);
      }
      // epilogue of output row 2h + pa: lane (lr, lh) holds channels cf * 16 + lh * 4 .. + 3 of
      // column w = m * 16 + lr (output column 2 (wl0 + w) + pb)
      const int Y = 2 * h + pa;
#pragma unroll
      for (int m = 0; m < 2; ++m) {
        float v[2][4];
#pragma unroll
        for (int cf = 0; cf < 2; ++cf)
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            v[cf][i] = acc[m][cf][i] + sbias[cg * 32 + cf * 16 + lh * 4 + i];
            st[cf][i] += v[cf][i];
            sq[cf][i] += v[cf][i] * v[cf][i];
          }
        const auto s0 = __builtin_amdgcn_permlane16_swap(pk(v[0][0], v[0][1]), pk(v[1][0], v[1][1]), false, false);
        const auto s1 = __builtin_amdgcn_permlane16_swap(pk(v[0][2], v[0][3]), pk(v[1][2], v[1][3]), false, false);
        const int X = 2 * (wl0 + m * 16 + lr) + pb;
        bf16* yp = reinterpret_cast<bf16*>(a.y) + ((long)(n * a.Ho + Y) * a.Wo + X) * a.ldy + cw + (lh & 1) * 16 +
                   (lh >> 1) * 8;
        *reinterpret_cast<uint4*>(yp) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
      }
    }
    if (a.stats && (it % UPB_G) == UPB_G - 1) {
      // record (block, 4-iteration group, phase): lanes 0-3 of a 16-lane row store the 4 channel
      // sums, lanes 4-7 the squares (conv_epilogue's record layout)
      const int rec = rec0 + (it / UPB_G) * 4 + ph;
#pragma unroll
      for (int cf = 0; cf < 2; ++cf) {
        float sv[4], qv[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          sv[i] = row16_sum(st[cf][i]);
          qv[i] = row16_sum(sq[cf][i]);
          st[cf][i] = sq[cf][i] = 0.f;
        }
        const int cb = cw + cf * 16 + lh * 4, ii = lr & 3;
        const float s01 = ii & 1 ? sv[1] : sv[0], s23 = ii & 1 ? sv[3] : sv[2];
        const float q01 = ii & 1 ? qv[1] : qv[0], q23 = ii & 1 ? qv[3] : qv[2];
        const float val = lr < 4 ? (ii & 2 ? s23 : s01) : (ii & 2 ? q23 : q01);
        if (lr < 8 && rec < a.nrec) a.stats[(long)(rec * 2 + (lr >> 2)) * a.Cout + cb + ii] = val;
      }
    }
  }
}

// ----------------------------------------------------------------------------------------
// 1x1 conv as a pixel stream: AFE.mid_conv 256 -> 512 (models.py:934) and Generator.mid_conv
// 256 -> 256 (models.py:1096) forward, and their data gradients (the same GEMM with the
// transposed weights, K = Cout).  out[p][co] = bias[co] + sum_k x[p][k] W[co][k]: per output
// pixel 2 K bytes in and 2 Cout bytes out for 2 K Cout FLOP, so at K <= 512 the launch is
// HBM-bound (conv_fwd_v2's 256 x 256 tile, one block per CU, alternated load -> MFMA -> store
// phases across the whole chip: 3.4 TB/s).
// A block owns 256 output channels; wave w keeps rows [32 w, 32 w + 32) of W for the whole
// launch as MFMA A fragments in registers (K / 4 VGPRs) and the block walks pixel tiles of
// BP = 16384 / K pixels (32 KB of x) persistently.  The x tiles land by LDS-DMA in a 4-slot
// ring, 3 tiles in flight while one is computed (with 2 slots of 64 KB only one tile was in
// flight per CU: 3.3 TB/s); the staged epilogue's stores of tile t drain under the DMA of
// tile t + 4, issued into the slot tile t just freed.  LDS rows are K * 2 bytes with the 16-B chunks XOR-swizzled by (pixel & 15)
// through the per-lane DMA source, so a fragment read (16 pixels at one k) is conflict-free.
// Co groups of one pixel stream are neighbouring blocks of one XCD (x read once into its L2).
// Requires P % BP == 0, Cout % 256 == 0, dense NHWC (ldy = Cout), no residual / statistics.
// ----------------------------------------------------------------------------------------
template <int K, int BPX>
__global__ void __launch_bounds__(512, 1)
conv1x1_stream(ConvArgs a, unsigned x_bytes) {
  constexpr int ROWB = K * 2, BP = BPX, RM = BP / 16, RN = 2, NKS = K / 32;
  constexpr int SLOT = BP * ROWB;                   // 32 / 64 KB
  constexpr int NSL = 131072 / SLOT;                // ring slots in 128 KB: NSL - 1 tiles in flight
  constexpr int PPW = SLOT / 1024 / 8;              // DMA pieces per wave per tile
  constexpr int RPP = 1024 / ROWB;                  // pixel rows per piece (2 / 1)
  constexpr int NST = RM;                           // 16-B output stores per lane per tile
  static_assert(K == 256 || K == 512, "conv1x1_stream: K of 256 or 512");
  static_assert(NSL >= 2 && NSL <= 4 && (NSL - 1) * PPW + NSL * NST <= 63, "conv1x1_stream: ring / vmcnt");
  __shared__ __attribute__((aligned(1024))) char smem[NSL * SLOT];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int lr = lane & 15, lh = lane >> 4;
  const int ncg = a.Cout / 256;
  const int bid = blockIdx.x, G = gridDim.x;
  const int cg = (bid / 8) % ncg;                   // the co groups of a stream share an XCD
  const int stream = bid % 8 + 8 * ((bid / 8) / ncg), nstream = G / ncg;
  const int co0 = cg * 256;
  const int ntp = a.P / BP;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);
  // lane part of a DMA piece: byte l * 16 of the piece = (row l / (64 / RPP), physical chunk);
  // the source is logical chunk (physical ^ (pixel & 15)); the piece's pixel offset & 15 is
  // RPP * (wave + 8 i) & 15: constant over i for RPP = 2, alternating for RPP = 1
  unsigned voff[2];
#pragma unroll
  for (int par = 0; par < 2; ++par) {
    const int rip = lane / (64 / RPP), pc = lane % (64 / RPP);
    const int prow = (RPP * (wave + 8 * par) + rip) & 15;
    voff[par] = (unsigned)((rip * K + ((pc ^ prow) << 3)) * 2);
  }
  // tile t into `slot`; t >= ntp issues the same pieces out of range (zero fill, no branch:
  // a branch here made the compiler keep live arrays in scratch across it)
  auto issue = [&](int t, int slot) {
    const unsigned base = sbase + slot * SLOT;
    const bool ok = t < ntp;
#pragma unroll
    for (int i = 0; i < PPW; ++i) {
      const int q = wave + 8 * i;
      dma16s(xr, base + q * 1024, ok ? voff[RPP == 2 ? 0 : (i & 1)] : 0x80000000u,
             ok ? (unsigned)(((t * BP + q * RPP) * K) * 2) : 0u);
    }
  };
  // this wave's weights: rows co0 + 32 wave + 16 n + lr, k = 32 s + 8 lh .. + 7
  Frag<bf16> wa[NKS][RN];
  {
    const bf16* w = reinterpret_cast<const bf16*>(a.w);
#pragma unroll
    for (int ss = 0; ss < NKS; ++ss)
#pragma unroll
      for (int n = 0; n < RN; ++n)
        wa[ss][n].v = *reinterpret_cast<const bf16x8*>(w + (long)(co0 + 32 * wave + 16 * n + lr) * a.Kpad + 32 * ss + 8 * lh);
  }
  // this lane's biases (channels co0 + 32 wave + 16 n + 4 lh + i), for every tile
  float bv[RN][4];
#pragma unroll
  for (int n = 0; n < RN; ++n)
#pragma unroll
    for (int i = 0; i < 4; ++i) bv[n][i] = a.bias ? a.bias[co0 + 32 * wave + 16 * n + 4 * lh + i] : 0.f;
  // fragment read of k-step s, m-tile m: pixel m * 16 + lr, physical chunk (4 s + lh) ^ lr
  unsigned foff[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) foff[q] = (unsigned)(lr * ROWB + (((4 * q + lh) ^ lr) << 4));
  auto pk = [](float lo, float hi) {
    const bf16 t2[2] = {(bf16)lo, (bf16)hi};
    return *reinterpret_cast<const unsigned*>(t2);
  };
  bf16* const yw = reinterpret_cast<bf16*>(a.y) + co0 + 32 * wave + (lh & 1) * 16 + (lh >> 1) * 8;

  int t = stream;
  if (t >= ntp) return;
#pragma unroll
  for (int j = 0; j < NSL; ++j) issue(t + j * nstream, j);
  for (int i = 0; t < ntp; t += nstream, ++i) {
    const int slot = i % NSL;
    // tile t landed: every wave waits for its own pieces, the barrier publishes them.  Issued
    // after tile t's pieces, in order: the prologue's later tiles, then per finished tile u the
    // pieces of tile u + NSL (zero-fill past the last tile) and u's stores -- exactly
    // (NSL - 1) x PPW pieces and min(i, NSL) x NST stores
    const int ni = i < NSL ? i : NSL;
    if (ni == 0) wait_vm<(NSL - 1) * PPW>();
    else if (ni == 1) wait_vm<(NSL - 1) * PPW + NST>();
    else if (ni == 2) wait_vm<(NSL - 1) * PPW + 2 * NST>();
    else if (ni == 3) wait_vm<(NSL - 1) * PPW + 3 * NST>();
    else wait_vm<(NSL - 1) * PPW + 4 * NST>();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    f32x4 acc[RN][RM];
#pragma unroll
    for (int n = 0; n < RN; ++n)
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[n][m] = f32x4{0.f, 0.f, 0.f, 0.f};
    const char* xs = smem + slot * SLOT;
    // two fragment sets: k-step ss + 1's reads under k-step ss's MFMAs; the scheduling
    // barriers keep the compiler from hoisting every k-step's reads (all of them in flight
    // spilled ~54 registers beside the resident weights)
    Frag<bf16> f0[RM], f1[RM];
    auto rd = [&](Frag<bf16> (&f)[RM], int ss) {
#pragma unroll
      for (int m = 0; m < RM; ++m) f[m].lds(xs + foff[ss & 3] + (ss >> 2) * 256 + m * 16 * ROWB);
    };
    auto mm = [&](const Frag<bf16> (&f)[RM], int ss) {
#pragma unroll
      for (int m = 0; m < RM; ++m)
#pragma unroll
        for (int n = 0; n < RN; ++n) acc[n][m] = mma(wa[ss][n], f[m], acc[n][m]);
    };
    rd(f0, 0);
#pragma unroll
    for (int ss = 0; ss < NKS; ss += 2) {
      rd(f1, ss + 1);
      __builtin_amdgcn_sched_barrier(0);
      mm(f0, ss);
      __builtin_amdgcn_sched_barrier(0);
      if (ss + 2 < NKS) rd(f0, ss + 2);
      __builtin_amdgcn_sched_barrier(0);
      mm(f1, ss + 1);
      __builtin_amdgcn_sched_barrier(0);
    }
    // every wave's fragment reads of the slot are done: refill it with tile t + NSL at once,
    // then the stores of tile t straight from the accumulators -- + bias, bf16, the two
    // 16-channel n-tiles paired by v_permlane16_swap so lane (lr, lh) holds 8 contiguous
    // channels ((lh & 1) * 16 + (lh >> 1) * 8 of the wave's 32) of pixel m * 16 + lr: one
    // 16-B store per m-tile (4 lanes = one 64-B channel run of a pixel)
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    issue(t + NSL * nstream, slot);
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const f32x4 va = acc[0][m], vb = acc[1][m];
      const auto s0 = __builtin_amdgcn_permlane16_swap(pk(va[0] + bv[0][0], va[1] + bv[0][1]),
                                                       pk(vb[0] + bv[1][0], vb[1] + bv[1][1]), false, false);
      const auto s1 = __builtin_amdgcn_permlane16_swap(pk(va[2] + bv[0][2], va[3] + bv[0][3]),
                                                       pk(vb[2] + bv[1][2], vb[3] + bv[1][3]), false, false);
      *reinterpret_cast<uint4*>(yw + (long)(t * BP + m * 16 + lr) * a.ldy) = make_uint4(s0[0], s1[0], s0[1], s1[1]);
    }
  }
  wait_vm<0>();      // the zero-fill pieces of the last tiles land before the workgroup's LDS is freed
}

// ----------------------------------------------------------------------------------------
// 7x7 conv with a 64-channel input and <= 4 output channels (Generator.out_conv 64 -> 3,
// models.py:1099 + sigmoid 1110), "column taps in N": for every input pixel w' of a row the
// block computes D[h][w'][(co, s)] = sum_{r, ci} x[h + r - 3][w'][ci] * W[co][ci][r][s]
// (M = pixels incl. the 3-pixel column halo, N = co x 7 taps = 21 of 32, K = 7 rows x 64 ci
// = 448), then out[h][w][co] = bias + sum_s D[h][w + s - 3][(co, s)].  3.5x fewer MFMAs than
// padding N = 3 to 16 with K = 3136, and each A fragment feeds two n-tiles.
// Block: TR = 4 output rows x 64 columns, 8 waves; halo [10 rows][70 cols][64 ci] in LDS.
// Wave w: row w >> 1 and five (m-tile, n-tile) pairs of that row's 5 m-tiles x 2 n-tiles.
// Weights wn [32][448] (n = co * 7 + s, k = r * 64 + ci, 28 KB) are staged in LDS with the halo.
// ----------------------------------------------------------------------------------------
constexpr int C7_TR = 4;   // output rows per band step of conv7_n3_fwd2 (H % C7_TR == 0)

// ----------------------------------------------------------------------------------------
// conv7_n3_fwd2: the "column taps in N" out_conv forward, sliding down a band of rows.
// (Its per-tile predecessor staged a 10-row halo for every 4 output rows: 2.5x input re-read,
// 598 MB of HBM per launch for a 268 MB input, one block per CU; 189 -> 118 us.)  Here a block
// owns (image, 64-column strip, band of C7B_BAND output rows) and keeps a ring of 14 input
// rows in LDS (72 pixels x 128 B = 9 pieces of 1 KB per row, so a row is whole DMA pieces):
// while the 8 waves compute output rows 4j..4j+3 from ring rows 4j-3..4j+6, the DMA of rows
// 4j+7..4j+10 (the next group's) is in flight.  Input bytes per launch ~1.05x the tensor.
// The weights sit in registers as MFMA B fragments (14 k-steps x 2 n-tiles, 112 VGPRs).
// Per group: D[row][w'][n] (fp32, the 21 used columns) through LDS, then the 7-tap column
// sums + bias (+ sigmoid, + BN records).
// ----------------------------------------------------------------------------------------
constexpr int C7B_SLOTS = 14, C7B_ROWPX = 72, C7B_ROWB = C7B_ROWPX * 128;   // 9216 B
constexpr int C7B_DLD = 22;                                                // D row stride (floats)
__global__ void __launch_bounds__(512, 1)
conv7_n3_fwd2(ConvArgs a, unsigned x_bytes, int band) {
  constexpr int RING = C7B_SLOTS * C7B_ROWB;                // 129024
  constexpr int DB = C7_TR * 70 * C7B_DLD * 4;               // 24640
  __shared__ __attribute__((aligned(1024))) char smem[RING + DB];
  float* Dl = reinterpret_cast<float*>(smem + RING);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int tiles_w = a.W / 64, bands = a.H / band;
  const int blk = blockIdx.x;
  const int n = blk / (bands * tiles_w);
  const int rem = blk - n * bands * tiles_w;
  const int hb = (rem / tiles_w) * band, w0 = (rem % tiles_w) * 64;
  const int li = lane & 15, g = lane >> 4;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);

  // ring row `rel` (input row hb - 3 + rel) -> slot rel % 14; 9 pieces per row
  auto issue_rows = [&](int rel0, int nrows) {
    for (int q = wave; q < nrows * 9; q += 8) {
      const int rr = q / 9, pc = q - rr * 9;
      const int rel = rel0 + rr;
      const int hh = hb - 3 + rel;
      const int L = pc * 64 + lane;                 // chunk within the row
      const int px = L >> 3, ch = L & 7;
      const int ww = w0 - 3 + px;
      const bool ok = px < 70 && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      // 16-B chunk swizzle by (px >> 1) & 7: 16 consecutive pixels (one fragment read) land on 16
      // different bank slots (by px & 7, pixels 8 apart shared one: 14 % bank conflicts)
      const unsigned off = ok ? (unsigned)((((n * a.H + hh) * a.W + ww) * 64 + ((ch ^ ((px >> 1) & 7)) << 3)) * 2)
                              : 0x80000000u;
      dma16(xr, smem + (rel % C7B_SLOTS) * C7B_ROWB + pc * 1024, off);
    }
  };
  issue_rows(0, 10);

  // weights wn [32][448] bf16 -> B fragments in registers
  const bf16* __restrict__ wn = reinterpret_cast<const bf16*>(a.w);
  bf16x8 bw[14][2];
#pragma unroll
  for (int ks = 0; ks < 14; ++ks)
#pragma unroll
    for (int t = 0; t < 2; ++t) bw[ks][t] = *reinterpret_cast<const bf16x8*>(wn + (t * 16 + li) * 448 + (ks * 4 + g) * 8);

  const int row = wave >> 1, half = wave & 1;
  const int mb = half ? 2 : 0;
  int apix[3];
#pragma unroll
  for (int t = 0; t < 3; ++t) apix[t] = min((mb + t) * 16 + li, C7B_ROWPX - 1);
  const int pm[5] = {half ? 2 : 0, half ? 3 : 0, half ? 3 : 1, half ? 4 : 1, half ? 4 : 2};
  const int pn[5] = {half ? 1 : 0, half ? 0 : 1, half ? 1 : 0, half ? 0 : 1, half ? 1 : 0};
  const int HWo = a.H * a.W;
  const int ngroups = band / C7_TR;
  float bias4[4];
#pragma unroll
  for (int c = 0; c < 4; ++c) bias4[c] = (a.bias && c < a.Cout) ? a.bias[c] : 0.f;
  // the epilogue's store instructions per group of this wave (lane 0's two record stores per
  // output too when statistics are on): the wait at the next group's top leaves them in flight
  // (it was vmcnt(0): every group waited for the previous group's output stores)
  const int nout = C7_TR * 64 * a.Cout;
  const int nst = (nout > wave * 64 ? (nout - wave * 64 + 511) / 512 : 0) * (a.stats ? 3 : 1);

  for (int j = 0; j < ngroups; ++j) {
    // group j's rows (issued at group j - 1's top; only this wave's stores of group j - 1 are
    // younger) landed for this wave; the barrier publishes every wave's and retires group
    // j - 1's D reads
    if (j == 0) wait_vm<0>();
    else wait_vm_dyn(nst);
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if (j + 1 < ngroups) issue_rows(4 * j + 10, 4);
    f32x4 acc[5];
#pragma unroll
    for (int i = 0; i < 5; ++i) acc[i] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int r = 0; r < 7; ++r) {
      const char* slot = smem + ((4 * j + row + r) % C7B_SLOTS) * C7B_ROWB;
#pragma unroll
      for (int kh = 0; kh < 2; ++kh) {
        const int ks = r * 2 + kh, c = kh * 4 + g;
        bf16x8 afr[3];
#pragma unroll
        for (int t = 0; t < 3; ++t)
          afr[t] = *reinterpret_cast<const bf16x8*>(slot + (apix[t] * 8 + (c ^ ((apix[t] >> 1) & 7))) * 16);
        if (half == 0) {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[0], bw[ks][0], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[0], bw[ks][1], acc[1], 0, 0, 0);
          acc[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[1], bw[ks][0], acc[2], 0, 0, 0);
          acc[3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[1], bw[ks][1], acc[3], 0, 0, 0);
          acc[4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[2], bw[ks][0], acc[4], 0, 0, 0);
        } else {
          acc[0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[0], bw[ks][1], acc[0], 0, 0, 0);
          acc[1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[1], bw[ks][0], acc[1], 0, 0, 0);
          acc[2] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[1], bw[ks][1], acc[2], 0, 0, 0);
          acc[3] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[2], bw[ks][0], acc[3], 0, 0, 0);
          acc[4] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[2], bw[ks][1], acc[4], 0, 0, 0);
        }
      }
    }
    // D[row][w'][n]: pixel w' = m*16 + 4g + i (MFMA row), column n = nt*16 + li; keep n < 21, w' < 70
#pragma unroll
    for (int i = 0; i < 5; ++i) {
      const int nn = pn[i] * 16 + li;
      if (nn < 21) {
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int wp = pm[i] * 16 + g * 4 + q;
          if (wp < 70) Dl[(row * 70 + wp) * C7B_DLD + nn] = acc[i][q];
        }
      }
    }
    wait_lgkm0();                              // D written (LDS only: the row DMA stays in flight)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    const int h0 = hb + 4 * j;
    for (int o = tid; o < nout; o += 512) {
      const int co = o / (C7_TR * 64), rr = (o / 64) % C7_TR, w = o % 64;
      float v = co == 0 ? bias4[0] : co == 1 ? bias4[1] : co == 2 ? bias4[2] : bias4[3];
#pragma unroll
      for (int s7 = 0; s7 < 7; ++s7) v += Dl[(rr * 70 + w + s7) * C7B_DLD + co * 7 + s7];
      if (a.stats) {
        const float sv = wave_sum(v), qv = wave_sum(v * v);
        const int rec = ((n * a.H + h0 + rr) * a.W + w0) >> 6;
        if (lane == 0 && rec < a.nrec) {
          a.stats[(long)(rec * 2) * a.Cout + co] = sv;
          a.stats[(long)(rec * 2 + 1) * a.Cout + co] = qv;
        }
      }
      if (a.sigmoid) v = 1.f / (1.f + expf(-v));
      const int pix = (h0 + rr) * a.W + w0 + w;
      if (a.nchw) reinterpret_cast<float*>(a.y)[((long)(n * a.Cout + co)) * HWo + pix] = v;
      else reinterpret_cast<bf16*>(a.y)[((long)n * HWo + pix) * a.ldy + co] = (bf16)v;
    }
  }
}

// wn [32][448]: n = co * 7 + s (co < cout, s < 7), k = r * 64 + ci
__global__ void weight_prep_c7n_kernel(const float* __restrict__ wp, const float* sigma, bf16* wn, int cout) {
  const float inv = sigma ? 1.f / sigma[0] : 1.f;
  for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < 32 * 448; e += gridDim.x * blockDim.x) {
    const int nn = e / 448, k = e - nn * 448;
    const int co = nn / 7, s = nn - co * 7, r = k >> 6, ci = k & 63;
    const float v = co < cout ? wp[((co * 64 + ci) * 7 + r) * 7 + s] * inv : 0.f;
    wn[e] = (bf16)v;
  }
}

// ----------------------------------------------------------------------------------------
// backward-weight:  D[k][co] = sum_p im2col(x)[p][k] * dy[p][co], split over pixels
// MFMA A operand = im2col^T (rows = k), B operand = dy (cols = co); both are k-slot =
// pixel, i.e. COLUMN reads of the [pixel][channel] LDS images -> ds_read_b64_tr_b16.
// ----------------------------------------------------------------------------------------
struct WgArgs {
  const void* x;
  const float* psc;
  const float* psh;
  float slope;
  const void* dy;
  float* slab;
  float* bslab;
  int N, H, W, Hin, Win, P;
  int lgCin, Cin;
  int K, KW;          // KW = slab row stride (>= Kpad, multiple of the k tile)
  int Cout, ldd;      // valid output channels, channel stride of dy
  int CW;             // slab co rows
  int ntk, ntc, steps_per_split, nsteps;
};

// 8-B granule swizzle for the transposed-read images (cols >= 64): conflict-free
// ds_read_b64_tr_b16 over rows {8g+q} (wgrad).
__device__ __forceinline__ int gswz(int row) { return (((row >> 1) & 1) | (((row >> 3) & 1) << 1)) << 2; }

template <int COLS>
__device__ __forceinline__ int tr_off(int row, int col) {  // byte offset of (row, col) bf16
  if constexpr (COLS >= 64) return row * COLS * 2 + (((col >> 2) ^ gswz(row)) << 3) + (col & 3) * 2;
  else return row * COLS * 2 + col * 2;
}

template <typename T, int COLS>
__device__ __forceinline__ void colfrag(const char* base, int cbase, int lane, Frag<T>& f) {
  const int g = lane >> 4, li = lane & 15;
  if constexpr (sizeof(T) == 2) {
    const int q = li >> 2, pp = li & 3;
    const int c = cbase + 4 * pp;
    FV_LDS char* lb = (FV_LDS char*)(base);   // generic -> LDS address-space cast
    s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + tr_off<COLS>(8 * g + q, c)));
    s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + tr_off<COLS>(8 * g + 4 + q, c)));
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    f.v = __builtin_bit_cast(bf16x8, v);
  } else {
    const float* fb = reinterpret_cast<const float*>(base);
#pragma unroll
    for (int j = 0; j < 8; ++j) f.v[j] = fb[(8 * g + j) * COLS + cbase + li];
  }
}

template <typename T, int KS, int WK, int WC, int RK, int RC, bool PRO, bool UPS>
__global__ void __launch_bounds__(64 * WK * WC)
conv_wgrad_kernel(WgArgs a) {
  constexpr int NT = 64 * WK * WC;
  constexpr int BKT = WK * RK * 16;  // k columns per block
  constexpr int BC = WC * RC * 16;   // output channels per block
  constexpr int PAD = KS / 2;
  constexpr int ES = sizeof(T);
  constexpr int PX = 32;             // pixels per step
  constexpr int ABYTES = PX * BKT * ES, DBYTES = PX * BC * ES;
  constexpr int KCH = BKT / 8, CCH = BC / 8;     // 8-element chunks per row
  constexpr int CA = (PX * KCH + NT - 1) / NT;
  constexpr int CD = (PX * CCH + NT - 1) / NT;
  static_assert(NT % KCH == 0 && NT % CCH == 0, "chunk map");
  __shared__ __attribute__((aligned(16))) char smem[2 * (ABYTES + DBYTES)];

  const T* __restrict__ x = reinterpret_cast<const T*>(a.x);
  const T* __restrict__ dy = reinterpret_cast<const T*>(a.dy);
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wk = wave % WK, wc = wave / WK;
  const int per = a.ntk * a.ntc;
  const int split = blockIdx.x / per;
  const int rem = blockIdx.x - split * per;
  const int tc = rem % a.ntc, tk = rem / a.ntc;
  const int k0 = tk * BKT, c0 = tc * BC;
  const int s_begin = split * a.steps_per_split;
  const int s_end = min(a.nsteps, s_begin + a.steps_per_split);
  const int HW = a.H * a.W;

  // fixed per-thread k chunk (gather) and co chunk (dy)
  const int kq = tid % KCH;
  const int kk = k0 + kq * 8;
  const bool kin = kk < a.K;
  const int tap = kk >> a.lgCin, ci = kk & (a.Cin - 1);
  const int rr = tap / KS, ss = tap - (tap / KS) * KS;
  const int cq = tid % CCH;
  const int cc = c0 + cq * 8;
  const bool cin_ok = cc < a.ldd;

  Chunk8<T> ra[CA], rd[CD];
  unsigned okm = 0;

  auto gload = [&](int st) {
    const int pbase = st * PX;
    okm = 0;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int q = tid + i * NT;
      const int prow = q / KCH;
      const int pix = pbase + prow;
      bool ok = kin && (q < PX * KCH) && pix < a.P;
      int n = pix / HW, r2 = pix - n * HW;
      int h = r2 / a.W, w = r2 - h * a.W;
      int hh = h + rr - PAD, ww = w + ss - PAD;
      int hs, ws;
      if constexpr (UPS) {
        ok = ok && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
        hs = hh >> 1;
        ws = ww >> 1;
      } else {
        ok = ok && hh >= 0 && hh < a.Hin && ww >= 0 && ww < a.Win;
        hs = hh;
        ws = ww;
      }
      if (ok) {
        ra[i].load(x + ((long)(n * a.Hin * a.Win + hs * a.Win + ws) << a.lgCin) + ci);
        okm |= 1u << i;
      } else {
        ra[i].zero();
      }
    }
#pragma unroll
    for (int i = 0; i < CD; ++i) {
      const int q = tid + i * NT;
      const int pix = pbase + q / CCH;
      if (cin_ok && q < PX * CCH && pix < a.P) rd[i].load(dy + (long)pix * a.ldd + cc);
      else rd[i].zero();
    }
  };

  auto chunk_off = [&](int row, int col, int cols) -> int {  // byte offset of an 8-elt chunk
    if constexpr (ES == 2) {
      if (cols >= 64) return row * cols * 2 + (((col >> 2) ^ gswz(row)) << 3);
      return row * cols * 2 + col * 2;
    } else {
      return (row * cols + col) * 4;
    }
  };

  auto lstore = [&](int buf) {
    char* As = smem + buf * (ABYTES + DBYTES);
    char* Ds = As + ABYTES;
#pragma unroll
    for (int i = 0; i < CA; ++i) {
      const int q = tid + i * NT;
      if (q < PX * KCH) {
        Chunk8<T> c = ra[i];
        if constexpr (PRO) {
          if (okm & (1u << i)) {
            float f[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) f[j] = fv_act(c.get(j) * a.psc[ci + j] + a.psh[ci + j], a.slope);
            c.set8(f);
          }
        }
        c.store(reinterpret_cast<T*>(As + chunk_off(q / KCH, kq * 8, BKT)));
      }
    }
#pragma unroll
    for (int i = 0; i < CD; ++i) {
      const int q = tid + i * NT;
      if (q < PX * CCH) rd[i].store(reinterpret_cast<T*>(Ds + chunk_off(q / CCH, cq * 8, BC)));
    }
  };

  f32x4 acc[RK][RC];
#pragma unroll
  for (int i = 0; i < RK; ++i)
#pragma unroll
    for (int j = 0; j < RC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // bias-gradient partial (only the k-tile-0 blocks): thread -> column tid % BC
  const bool do_bias = (tk == 0) && a.bslab;
  constexpr int BROWS = NT / BC > 0 ? NT / BC : 1;
  float bsum = 0.f;

  auto compute = [&](int buf) {
    const char* As = smem + buf * (ABYTES + DBYTES);
    const char* Ds = As + ABYTES;
    Frag<T> af[RK], bfr[RC];
#pragma unroll
    for (int i = 0; i < RK; ++i) colfrag<T, BKT>(As, wk * RK * 16 + i * 16, lane, af[i]);
#pragma unroll
    for (int j = 0; j < RC; ++j) colfrag<T, BC>(Ds, wc * RC * 16 + j * 16, lane, bfr[j]);
#pragma unroll
    for (int i = 0; i < RK; ++i)
#pragma unroll
      for (int j = 0; j < RC; ++j) acc[i][j] = mma(af[i], bfr[j], acc[i][j]);
    if (do_bias && tid < BROWS * BC) {
      const int col = tid % BC, part = tid / BC;
      for (int r = part; r < PX; r += BROWS) {
        if constexpr (ES == 2) bsum += (float)*reinterpret_cast<const bf16*>(Ds + tr_off<BC>(r, col));
        else bsum += reinterpret_cast<const float*>(Ds)[r * BC + col];
      }
    }
  };

  if (s_begin < s_end) {
    gload(s_begin);
    lstore(0);
    __syncthreads();
    for (int st = s_begin; st < s_end; ++st) {
      const int cur = (st - s_begin) & 1;
      if (st + 1 < s_end) gload(st + 1);
      compute(cur);
      if (st + 1 < s_end) lstore(cur ^ 1);
      __syncthreads();
    }
  }

  // D[k][co]: lane holds k = kb + 4*(lane>>4) + i for co = cb + (lane & 15)
  const int lr = lane & 15, lh = lane >> 4;
  float* slab = a.slab + (long)split * a.CW * a.KW;
#pragma unroll
  for (int i = 0; i < RK; ++i) {
    const int kb = k0 + wk * RK * 16 + i * 16 + lh * 4;
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      const int co = c0 + wc * RC * 16 + j * 16 + lr;
      *reinterpret_cast<float4*>(slab + (long)co * a.KW + kb) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
  if (do_bias) {
    float* red = reinterpret_cast<float*>(smem);
    if (tid < BROWS * BC) red[tid] = bsum;
    __syncthreads();
    if (tid < BC) {
      float t = 0.f;
      for (int p = 0; p < BROWS; ++p) t += red[p * BC + tid];
      a.bslab[(long)split * a.CW + c0 + tid] = t;
    }
  }
}

// ----------------------------------------------------------------------------------------
// backward-weight v2 (bf16): D[k][co] = sum_p im2col(x)[p][k] * dy[p][co] as a pixel-K GEMM.
// 8 waves, block tile BKT (k) x BC (co), PX pixels per stage, NS-stage LDS ring filled by
// buffer_load ... lds (the DMA destination is lane-linear, so the 32-B-block XOR swizzle
// that makes the transposed fragment reads conflict-free is applied to the SOURCE
// address), counted vmcnt + raw s_barrier so NS-1 stages stay in flight.  Fragments are
// read with ds_read_b64_tr_b16 (pixels are the MFMA K).  Zero padding (image border,
// k >= K, co >= ldd, pixel >= P) comes from the buffer range check (offset 0x80000000).
// The bias gradient sum_p dy[p][co] rides along as one extra MFMA per co tile with an
// all-ones A operand (k-tile-0 blocks, k-wave 0 only).  Output: per-split fp32 slabs.
// ----------------------------------------------------------------------------------------
struct Wg2Args {
  const void* x;
  const void* dy;
  float* slab;
  float* bslab;
  int H, W, Hin, Win, P;
  int lgCin, K, KW, ldd, CW;
  int ntk, ntc, nsteps, sps;
  FastDiv fhw, fw, fh;
  unsigned xbytes, dybytes;
  int rowal;   // W % PX == 0: each stage lies in one image row
  // sub-pixel phases of an upsample + 3x3 conv (SUB): pixels are the LOW-res image (H x W),
  // the block's phase (pa, pb) pairs low-res pixel (n, i, j) with dy pixel (n, 2i+pa, 2j+pb)
  // of the Ho x Wo image; phase slabs follow each other ([4][nsplit][CW][KW])
  int Ho, Wo, nsplit;
  int il;      // row-aligned stages: spread the next stage's DMA pieces between MFMAs
};

// 32-B-block XOR of a [row][NCOL] bf16 image: the 8 rows {0-3, 8-11} (and {4-7, 12-15}) one
// ds_read_b64_tr_b16 lane group touches land on 8 distinct 32-B bank slots.
template <int NCOL>
__device__ __forceinline__ int tswz(int row) {
  if constexpr (NCOL >= 128) return (row & 3) | (((row >> 3) & 1) << 2);
  else if constexpr (NCOL == 64) return ((row >> 1) & 1) | (((row >> 3) & 1) << 1);
  else if constexpr (NCOL == 32) return (row >> 3) & 1;   // rows r and r + 8 in different halves
  else return 0;
}
template <int NCOL>
__device__ __forceinline__ int timg_off(int row, int col) {  // col % 4 == 0
  return row * NCOL * 2 + ((((col >> 4) ^ tswz<NCOL>(row)) << 5) | ((col & 15) << 1));
}
// 16 columns x 32 rows (rows r0..r0+31) -> MFMA K-fragment of column (cbase + lane & 15)
template <int NCOL>
__device__ __forceinline__ bf16x8 tfrag(const char* base, int r0, int cbase, int lane) {
  const int g = lane >> 4, li = lane & 15;
  // NCOL < 16 (8 staged channels): lanes of columns >= NCOL re-read valid columns; the
  // caller ignores those outputs (every lane must take part in a transposed read)
  const int c = (cbase + 4 * (li & 3)) & (NCOL >= 16 ? ~0 : NCOL - 1);
  FV_LDS char* lb = (FV_LDS char*)(base);
  const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + timg_off<NCOL>(r0 + 8 * g + (li >> 2), c)));
  const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + timg_off<NCOL>(r0 + 8 * g + 4 + (li >> 2), c)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

template <int N>
__device__ __forceinline__ void wait_vmcnt() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory"); }

// ring wait: retire the oldest stage while `ahead` (0 .. NS-2, run-time) younger ones stay in flight
template <int NS, int PW, int A = NS - 2>  // vmcnt immediate <= 63: (NS - 2) * PW must fit
__device__ __forceinline__ void wait_ahead(int ahead) {
  if constexpr (A <= 0) {
    wait_vmcnt<0>();
  } else {
    if (ahead >= A) wait_vmcnt<A * PW>();
    else wait_ahead<NS, PW, A - 1>(ahead);
  }
}

template <int KS, int BKT, int BC, int WK, int WC, int PX, int NS, bool UPS, bool SUB = false>
__global__ void __launch_bounds__(512, 2)
conv_wgrad_v2(Wg2Args a) {
  static_assert(!SUB || (KS == 2 && !UPS), "sub-pixel wgrad: 2x2 taps, no upsample");
  static_assert(WK * WC == 8, "8 waves");
  constexpr int RK = BKT / (16 * WK), RC = BC / (16 * WC);
  static_assert(RK * 16 * WK == BKT && RC * 16 * WC == BC, "wave tiling");
  constexpr int PAD = KS / 2;
  constexpr int SA = PX * BKT * 2, SB = PX * BC * 2, STAGE = SA + SB;
  constexpr int QA = SA / 1024, QB = SB / 1024;            // 1-KB DMA pieces per stage
  static_assert(QA * 1024 == SA && QB * 1024 == SB, "pieces");
  constexpr int JA = (QA + 7) / 8, JB = (QB + 7) / 8;      // pieces per wave
  constexpr int PW = JA + JB;                              // upper bound of DMAs per wave per stage
  constexpr int CPA = BKT / 8, CPB = BC / 8;               // 16-B chunks per row
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wk = wave % WK, wc = wave / WK;
  // XCD-aware order: the blocks of one pixel split (all k/co tiles: same dy rows, overlapping
  // x rows) share an XCD's L2.  Bijective remap; speed only.
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int lid0 = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int phase = SUB ? (lid0 & 3) : 0;      // the 4 phases of a split are neighbours
  const int lid = SUB ? (lid0 >> 2) : lid0;
  const int pa = phase >> 1, pb = phase & 1;
  const int ntile = a.ntk * a.ntc;
  const int split = lid / ntile, tile = lid - split * ntile;
  const int tc = tile % a.ntc, tk = tile / a.ntc;
  const int k0 = tk * BKT, c0 = tc * BC;
  const int s_begin = split * a.sps;
  const int nst = min(a.nsteps, s_begin + a.sps) - s_begin;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dy), 0, (int)a.dybytes, 0x00020000);

  // per-piece constants: row in the stage image and the (tap, ci) of this lane's chunk
  int arow[JA], adh[JA], adw[JA], aci[JA];
  bool akin[JA];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int q = wave + j * 8;
    const int L = q * 64 + lane;
    const int row = L / CPA, dch = L % CPA;
    const int sc = (((dch >> 1) ^ tswz<BKT>(row)) << 1) | (dch & 1);
    const int k = k0 + sc * 8;
    const int tap = k >> a.lgCin;
    const int r = tap / KS, s = tap - (tap / KS) * KS;
    arow[j] = row;
    adh[j] = SUB ? r + pa - 1 : r - PAD;
    adw[j] = SUB ? s + pb - 1 : s - PAD;
    aci[j] = k & ((1 << a.lgCin) - 1);
    akin[j] = (QA % 8 == 0 || q < QA) && k < a.K;
  }
  int brow[JB], bco[JB];
  bool bok[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int q = wave + j * 8;
    const int L = q * 64 + lane;
    const int row = L / CPB, dch = L % CPB;
    const int sc = CPB >= 4 ? ((((dch >> 1) ^ tswz<BC>(row)) << 1) | (dch & 1)) : dch;
    brow[j] = row;
    bco[j] = c0 + sc * 8;
    bok[j] = (QB % 8 == 0 || q < QB) && bco[j] < a.ldd;
  }

  // row-aligned stages (W % PX == 0, so P % PX == 0 too): a stage is one image-row segment
  // (n, h, w0 wave-uniform).  The lane's part of its im2col source offset is precomputed
  // relative to (h, w0) -- per h parity when upsampling -- so a piece costs an add, two
  // range compares and a select; the dy pieces are a fixed per-lane offset + soffset.
  int cwA[JA], cA0[JA], cA1[JA];
#pragma unroll
  for (int j = 0; j < JA; ++j) {
    const int cw = akin[j] ? arow[j] + adw[j] : 0x40000000;   // column relative to w0
    cwA[j] = cw;
    if (UPS) {
      cA0[j] = (((((adh[j] >> 1) * a.Win) + (cw >> 1)) << a.lgCin) + aci[j]) * 2;
      cA1[j] = (((((1 + adh[j]) >> 1) * a.Win + (cw >> 1)) << a.lgCin) + aci[j]) * 2;
    } else {
      cA0[j] = cA1[j] = (((adh[j] * a.Win + cw) << a.lgCin) + aci[j]) * 2;
    }
  }
  unsigned cB[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) cB[j] = bok[j] ? (unsigned)(brow[j] * (SUB ? 2 : 1) * a.ldd + bco[j]) * 2u : 0x80000000u;
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);

  // row-aligned stage: wave-uniform state once per stage, then one DMA piece at a time, so
  // the pieces can be spread between MFMAs (a piece costs ~60 cycles among MFMAs, 100-185
  // back to back; issued as a block, both waves of a SIMD stall on them together)
  struct RowSt {
    unsigned As, Bs, dpo;
    int S, h, w0;
    bool sok, odd;
  };
  auto rowal_state = [&](int st, int buf) {
    RowSt r;
    const int pbase = (s_begin + st) * PX;
    r.As = sbase + buf * STAGE;
    r.Bs = r.As + SA;
    const int hrow = (int)fdiv((uint32_t)pbase, a.fw);
    r.w0 = pbase - hrow * a.W;
    const int n = (int)fdiv((uint32_t)hrow, a.fh);
    r.h = hrow - n * a.H;
    r.sok = pbase < a.P;
    r.S = UPS ? ((((n * a.Hin + (r.h >> 1)) * a.Win + (r.w0 >> 1)) << a.lgCin) * 2)
              : ((((n * a.Hin + r.h) * a.Win + r.w0) << a.lgCin) * 2);
    r.odd = UPS && (r.h & 1);
    // dy pixel of the stage's first pixel: itself, or (n, 2h+pa, 2*w0+pb) for a phase
    const unsigned dp = SUB ? (unsigned)((n * a.Ho + 2 * r.h + pa) * a.Wo + 2 * r.w0 + pb) : (unsigned)pbase;
    r.dpo = dp * (unsigned)a.ldd * 2u;
    return r;
  };
  // piece q in [0, JA + JB): x pieces first, then dy (compile-time q after unrolling)
  auto rowal_piece = [&](const RowSt& r, int q) {
    if (q < JA) {
      const int j = q, qq = wave + j * 8;
      if (QA % 8 == 0 || qq < QA) {
        const bool ok = r.sok && (unsigned)(r.h + adh[j]) < (unsigned)a.H && (unsigned)(r.w0 + cwA[j]) < (unsigned)a.W;
        const int c = r.odd ? cA1[j] : cA0[j];
        dma16s(xr, r.As + qq * 1024, ok ? (unsigned)(r.S + c) : 0x80000000u, 0u);
      }
    } else {
      const int j = q - JA, qq = wave + j * 8;
      if (QB % 8 == 0 || qq < QB) {
        if (r.sok) dma16s(dr, r.Bs + qq * 1024, cB[j], r.dpo);
        else dma16s(dr, r.Bs + qq * 1024, 0x80000000u, 0u);
      }
    }
  };
  auto issue_rowal = [&](int st, int buf) {
    const RowSt r = rowal_state(st, buf);
#pragma unroll
    for (int q = 0; q < JA + JB; ++q) rowal_piece(r, q);
  };

  auto issue = [&](int st, int buf) {
    if (SUB || a.rowal) {        // SUB: the host only launches row-aligned stages
      issue_rowal(st, buf);
      return;
    }
    const int pbase = (s_begin + st) * PX;
    char* As = smem + buf * STAGE;
    char* Bs = As + SA;
#pragma unroll
    for (int j = 0; j < JA; ++j) {
      const int q = wave + j * 8;
      if (QA % 8 == 0 || q < QA) {
        const int p = pbase + arow[j];
        const int n = (int)fdiv((uint32_t)p, a.fhw);
        const int rem = p - n * a.H * a.W;
        const int h = (int)fdiv((uint32_t)rem, a.fw);
        const int w = rem - h * a.W;
        const int hh = h + adh[j], ww = w + adw[j];
        bool ok = akin[j] && p < a.P && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
        const int hs = UPS ? (hh >> 1) : hh, ws = UPS ? (ww >> 1) : ww;
        const unsigned off = ok ? ((unsigned)(((n * a.Hin + hs) * a.Win + ws) << a.lgCin) + (unsigned)aci[j]) * 2u
                                : 0x80000000u;
        dma16(xr, As + q * 1024, off);
      }
    }
#pragma unroll
    for (int j = 0; j < JB; ++j) {
      const int q = wave + j * 8;
      if (QB % 8 == 0 || q < QB) {
        const int p = pbase + brow[j];
        const bool ok = bok[j] && p < a.P;
        const unsigned off = ok ? ((unsigned)p * (unsigned)a.ldd + (unsigned)bco[j]) * 2u : 0x80000000u;
        dma16(dr, Bs + q * 1024, off);
      }
    }
  };
  // a counted vmcnt needs every wave to issue exactly PW DMAs per stage
  static_assert((QA % 8 == 0 && QB % 8 == 0) || NS == 2, "uneven DMA split needs NS == 2 (vmcnt(0))");

  f32x4 acc[RK][RC];
#pragma unroll
  for (int i = 0; i < RK; ++i)
#pragma unroll
    for (int j = 0; j < RC; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.bslab && tk == 0 && wk == 0;
  f32x4 accb[RC];
#pragma unroll
  for (int j = 0; j < RC; ++j) accb[j] = f32x4{0.f, 0.f, 0.f, 0.f};
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;

  // hook(i): called after MFMA row i of the first 32-pixel slice (the DMA pieces of the
  // next stage go there)
  auto compute_h = [&](int buf, auto&& hook) {
    const char* As = smem + buf * STAGE;
    const char* Bs = As + SA;
#pragma unroll
    for (int kk = 0; kk < PX / 32; ++kk) {
      bf16x8 af[RK], bfr[RC];
#pragma unroll
      for (int j = 0; j < RC; ++j) bfr[j] = tfrag<BC>(Bs, kk * 32, wc * RC * 16 + j * 16, lane);
#pragma unroll
      for (int i = 0; i < RK; ++i) af[i] = tfrag<BKT>(As, kk * 32, wk * RK * 16 + i * 16, lane);
#pragma unroll
      for (int i = 0; i < RK; ++i) {
#pragma unroll
        for (int j = 0; j < RC; ++j) acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bfr[j], acc[i][j], 0, 0, 0);
        if (kk == 0) hook(i);
      }
      if (do_bias) {
#pragma unroll
        for (int j = 0; j < RC; ++j) accb[j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bfr[j], accb[j], 0, 0, 0);
      }
    }
  };

  // ring: NS-1 stages in flight; stage `it` is waited for with a counted vmcnt, then one
  // raw barrier publishes it (and retires every wave's reads of the buffer re-filled next).
#pragma unroll
  for (int i = 0; i < NS - 1; ++i)
    if (i < nst) issue(i, i);
  if ((SUB || a.rowal) && a.il) {
    // the next stage's pieces spread over the first slice's MFMA rows (all issued within the
    // iteration, in piece order: the counted waits are unchanged)
    for (int it = 0; it < nst; ++it) {
      const int ahead = min(NS - 2, nst - 1 - it);
      wait_ahead<NS, PW>(ahead);
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      const bool more = it + NS - 1 < nst;
      const RowSt r = rowal_state(it + NS - 1, (it + NS - 1) % NS);
      compute_h(it % NS, [&](int i) {
#pragma unroll
        for (int q = i * (JA + JB) / RK; q < (i + 1) * (JA + JB) / RK; ++q)
          if (more) rowal_piece(r, q);
      });
    }
  } else {
    for (int it = 0; it < nst; ++it) {
      const int ahead = min(NS - 2, nst - 1 - it);   // younger stages allowed in flight
      wait_ahead<NS, PW>(ahead);
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      if (it + NS - 1 < nst) issue(it + NS - 1, (it + NS - 1) % NS);
      compute_h(it % NS, [](int) {});
    }
  }

  // D[k][co]: lane holds k = kb + 4*(lane>>4) + i for co = cb + (lane & 15)
  const int lr = lane & 15, lh = lane >> 4;
  float* slab = a.slab + (long)(SUB ? phase * a.nsplit + split : split) * a.CW * a.KW;
#pragma unroll
  for (int i = 0; i < RK; ++i) {
    const int kb = k0 + wk * RK * 16 + i * 16 + lh * 4;
#pragma unroll
    for (int j = 0; j < RC; ++j) {
      const int co = c0 + wc * RC * 16 + j * 16 + lr;
      *reinterpret_cast<float4*>(slab + (long)co * a.KW + kb) =
          make_float4(acc[i][j][0], acc[i][j][1], acc[i][j][2], acc[i][j][3]);
    }
  }
  if (do_bias && lh == 0) {
#pragma unroll
    for (int j = 0; j < RC; ++j)
      a.bslab[(long)(SUB ? phase * a.nsplit + split : split) * a.CW + c0 + wc * RC * 16 + j * 16 + lr] = accb[j][0];
  }
}

// ----------------------------------------------------------------------------------------
// Sliding-row weight gradient of a 3x3 conv with 64 input channels (AFE.down1 64 -> 128 at
// full resolution), each operand byte read from HBM once: a block owns 128 co x ALL 9 taps x
// 64 ci (= 128 x 576, 36 accumulators per wave) and walks the rows [h0, h1) of one 64-column
// strip of one image.  Per row h it needs dy row h and x rows h-1, h, h+1; dy rows stream
// through a 3-deep ring, x rows through a 5-deep ring where each row lands once and stays for
// the three rows that read it (its tile-per-segment predecessor restaged dy per 32-channel
// k-tile and a fresh 3-row halo per segment: 2.76x the algorithmic bytes).  A "group" i = {dy row h0+i, x row
// h0+i+1} is issued two rows ahead; a wave's DMAs of a group are counted (wave 0 issues 4 of
// the 25 pieces, the others 3) so the wait for group i leaves group i+1 in flight.
//   8 waves = 2 (64 co) x 4 (9 of the 36 k-tiles of 16 = (tap, 16 ci)).
// Output: slab [block][cout][576] (k = tap * 64 + ci: wgrad_reduce_kernel's layout) and the
// bias slab [block][cout] (sum of dy by an all-ones MFMA operand, k-wave 0).
// ----------------------------------------------------------------------------------------
struct H3Wg2Args {
  const void* x;
  const void* dy;
  float* slab;
  float* bslab;
  int H, W, Cout, ldd, nseg, rows, nct;
  int ldx, nci;          // x channel stride (= Cin) and 64-channel input tiles (Cin / 64)
  unsigned xbytes, dybytes;
};

// (measured r5, not kept: one static s_setprio 1 for waves 4-7 instead of the per-half flips,
// and the second k-half's dy fragments read under the first half's last MFMA group -- res /
// down2 / down1 143 / 288 / 355 us either way, the prefetch variant spills at 256 VGPRs;
// profiles/r5/r5c_*)
template <int AHEAD>
__global__ void __launch_bounds__(512, 1)
conv3_halo_wgrad2(H3Wg2Args a) {
  // AHEAD groups in flight: group i + AHEAD is issued in row step i (HBM latency under load
  // is several row steps of MFMA work); rings: dy AHEAD + 1 deep, x AHEAD + 3 deep
  constexpr int XA = 1;                               // group i carries x row h0 + i + XA
  constexpr int BC = 128, NSD = AHEAD + 1, NSX = AHEAD + 2 + XA;
  constexpr int DYB = 64 * BC * 2;                    // 16 KB, 16 pieces
  constexpr int XQ = (66 * 128 + 1023) / 1024;        // 9 pieces per x row (66 px x 64 ci)
  constexpr int XB = XQ * 1024;
  constexpr int NPC = 16 + XQ;                        // pieces per group (25)
  __shared__ __attribute__((aligned(1024))) char smem[NSD * DYB + NSX * XB];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave & 1, wk = wave >> 1;
  const int li = lane & 15, g = lane >> 4;
  const int strips = a.W >> 6;
  // XCD-aware order (bijective remap, speed only): the nct x nci tiles of one (image, strip,
  // segment) -- the same dy and x rows -- are consecutive lids, dealt to one XCD's L2
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int ntile = a.nct * a.nci;
  const int tile = blk % ntile, tc = tile % a.nct, tci = tile / a.nct;
  const int split = blk / ntile;
  const int seg = split % a.nseg, strip = (split / a.nseg) % strips, n = split / (a.nseg * strips);
  const int co0 = tc * BC, w0 = strip * 64, ci0 = tci * 64;
  const int h0 = seg * a.rows, h1 = min(a.H, h0 + a.rows);
  const int nrow = h1 - h0;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dy), 0, (int)a.dybytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);

  // per-lane constants of this wave's pieces: piece q = wave + 8 j of a group (q < 16: dy,
  // else x piece q - 16); source offsets relative to the row start (0x80000000: outside)
  const int npw = wave == 0 ? 4 : 3;                  // pieces of a group this wave issues
  unsigned poff[4];
  int pisx[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const int q = wave + 8 * j;
    pisx[j] = q >= 16;
    if (q < 16) {
      const int o = q * 1024 + lane * 16;
      const int px = o / (BC * 2), b = o - px * (BC * 2);
      const int co = ((((b >> 5) ^ tswz<BC>(px)) << 4) | (((b >> 4) & 1) << 3));
      poff[j] = (unsigned)((px * a.ldd + co0 + co) * 2);          // + row base * ldd * 2
    } else if (q < NPC) {
      const int o = (q - 16) * 1024 + lane * 16;
      const int px = o >> 7, b = o & 127;
      const int ci = ((((b >> 5) ^ tswz<64>(px)) << 4) | (((b >> 4) & 1) << 3));
      const int iw = w0 - 1 + px;
      poff[j] = (px < 66 && iw >= 0 && iw < a.W) ? (unsigned)((iw * a.ldx + ci0 + ci) * 2) : 0x80000000u;
    } else {
      poff[j] = 0x80000000u;
    }
  }
  // x row y (image row, may be outside) -> ring slot (y - h0 + 1) % NSX; dy row h -> (h - h0) % NSD
  auto issue_x = [&](int y, int j) {          // the wave's j-th piece when it is an x piece
    const int slot = (y - h0 + 1) % NSX;
    const int q = wave + 8 * j - 16;
    const bool rok = y >= 0 && y < a.H;               // wave-uniform (the column test is in poff)
    dma16s(xr, sbase + NSD * DYB + slot * XB + q * 1024, rok ? poff[j] : 0x80000000u,
           rok ? (unsigned)(((n * a.H + y) * a.W) * a.ldx * 2) : 0u);
  };
  // pieces q = wave + 8 j: j = 0, 1 are dy pieces (q < 16), j = 2 the x piece wave, j = 3 x
  // piece 8 for wave 0 only (pisx / npw as compile-time structure: no per-piece branches)
  auto issue_group = [&](int i) {             // dy row h0 + i, x row h0 + i + XA
    const int h = h0 + i;
    const unsigned dbase = sbase + (i % NSD) * DYB;
    const unsigned drow = (unsigned)((((n * a.H + h) * a.W + w0) * a.ldd) * 2);
    dma16s(dr, dbase + wave * 1024, poff[0], drow);
    dma16s(dr, dbase + (wave + 8) * 1024, poff[1], drow);
    issue_x(h + XA, 2);
    if (wave == 0) issue_x(h + XA, 3);
  };
  auto issue_xonly = [&](int y) {             // prologue rows h0 - 1 .. h0 + XA - 1
#pragma unroll
    for (int j = 0; j < 4; ++j)
      if (j < npw && pisx[j]) issue_x(y, j);
  };

#pragma unroll
  for (int y = -1; y < XA; ++y) issue_xonly(h0 + y);
#pragma unroll
  for (int i = 0; i < AHEAD; ++i)
    if (i < nrow) issue_group(i);
  // the wave's k-wave index as a compile-time constant (its 9 k-tiles, and the bias MFMAs of
  // k-wave 0, then need no registers)
  with_const<0, 4>(wk, [&](auto wkc) {
    constexpr int WK = decltype(wkc)::value;
    constexpr bool BIAS_W = WK == 0;
    f32x4 acc[4][9];
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int j = 0; j < 9; ++j) acc[q][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    f32x4 accb[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) accb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
    const bool do_bias = BIAS_W && a.bslab && tci == 0;
    bf16x8 ones;
#pragma unroll
    for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;
    // transposed-read lane constants, hoisted out of the row loop: both images' swizzles have
    // a 16-row period and every fragment starts at kk * 32 (+ the tap column for x), so a
    // read's address is slot base + lane constant (per fragment and 4-row half) + an immediate
    // (the same addresses as tfrag: bit-identical)
    unsigned lcd[4][2], lcx[9][2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      const int rl = 8 * g + 4 * h + (li >> 2);
#pragma unroll
      for (int q = 0; q < 4; ++q) lcd[q][h] = (unsigned)timg_off<BC>(rl, wc * 64 + q * 16 + 4 * (li & 3));
#pragma unroll
      for (int j = 0; j < 9; ++j) {
        const int kt = 9 * WK + j, tap = kt >> 2;
        lcx[j][h] = (unsigned)timg_off<64>(tap % 3 + rl, (kt & 3) * 16 + 4 * (li & 3));
      }
    }
    typedef short s16x8 __attribute__((ext_vector_type(8)));
    auto frag2 = [](const char* base, unsigned l0, unsigned l1, int off) {
      FV_LDS char* lb = (FV_LDS char*)(base) + off;
      const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + l0));
      const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + l1));
      const s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
      return __builtin_bit_cast(bf16x8, v);
    };
    // ring slots of the step's dy row and x rows h - 1 .. h + 1, advanced with a wrap (scalar):
    // each read address is then lane constant + slot base (one add per distinct address and
    // step, the two k-halves by immediate offsets) -- the compiler's strength-reduced
    // (i + r) % NSX took ~100 vector adds per step (r6)
    int sd = 0, sx = 0;
    for (int i = 0; i < nrow; ++i) {
      // group i landed; the younger groups issued so far (up to AHEAD - 1) may stay in flight:
      // steady state 3 (AHEAD - 1) groups of npw pieces, counted at compile time per npw
      if (i + AHEAD - 1 < nrow) {
        if (npw == 4) wait_vm<4 * (AHEAD - 1)>();
        else wait_vm<3 * (AHEAD - 1)>();
      } else {
        wait_vm_dyn((nrow - 1 - i) * npw);
      }
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (i + AHEAD < nrow) issue_group(i + AHEAD);
      unsigned bd = (unsigned)(sd * DYB), bx[3];
#pragma unroll
      for (int r = 0; r < 3; ++r) {
        const int t = sx + r;
        bx[r] = (unsigned)(NSD * DYB + (t >= NSX ? t - NSX : t) * XB);
      }
      asm volatile("" : "+s"(bd), "+s"(bx[0]), "+s"(bx[1]), "+s"(bx[2]));
      sd = sd + 1 == NSD ? 0 : sd + 1;
      sx = sx + 1 == NSX ? 0 : sx + 1;
      unsigned ad[4][2], ax[9][2];
#pragma unroll
      for (int h = 0; h < 2; ++h) {
#pragma unroll
        for (int q = 0; q < 4; ++q) ad[q][h] = lcd[q][h] + bd;
#pragma unroll
        for (int j = 0; j < 9; ++j) ax[j][h] = lcx[j][h] + bx[((9 * WK + j) >> 2) / 3];
      }
      const char* const dys = smem;
      // x fragment of k-tile j of k-half kk (tap row / column constant after unrolling)
      auto xfrag = [&](int j, int kk) { return frag2(smem, ax[j][0], ax[j][1], kk * 32 * 128); };
#pragma unroll
      for (int kk = 0; kk < 2; ++kk) {
        bf16x8 af[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) af[q] = frag2(dys, ad[q][0], ad[q][1], kk * 32 * BC * 2);
        // the next x fragment is read before the current one's 4 MFMAs so the LDS latency hides
        // under them
        bf16x8 bcur = xfrag(0, kk);
        __builtin_amdgcn_s_setprio(1);
#pragma unroll
        for (int j = 0; j < 9; ++j) {
          bf16x8 bnext = bcur;
          if (j + 1 < 9) bnext = xfrag(j + 1, kk);
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[q], bcur, acc[q][j], 0, 0, 0);
          bcur = bnext;
        }
        if (do_bias) {
#pragma unroll
          for (int q = 0; q < 4; ++q) accb[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[q], ones, accb[q], 0, 0, 0);
        }
        __builtin_amdgcn_s_setprio(0);
      }
    }
    // slab[split][co][tap * Cin + ci]: lane holds D[co = 4g + jj][k-col = li]
    const long KW = 9L * a.ldx;
    float* sl = a.slab + (long)split * a.Cout * KW;
#pragma unroll
    for (int j = 0; j < 9; ++j) {
      const int kt = 9 * WK + j, tap = kt >> 2;
      const int kcol = tap * a.ldx + ci0 + (kt & 3) * 16 + li;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) sl[(long)(co0 + wc * 64 + q * 16 + 4 * g + jj) * KW + kcol] = acc[q][j][jj];
    }
    if (do_bias && li == 0) {
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          a.bslab[(long)split * a.Cout + co0 + wc * 64 + q * 16 + 4 * g + jj] = accb[q][jj];
    }
  });
}

// ----------------------------------------------------------------------------------------
// Sub-pixel weight gradient of the UpBlock2D convs (nearest x2 upsample + 3x3, modules.py:78-89;
// VERDICT r4 item 2) on the sliding-row structure of conv3_halo_wgrad2: output row Y = 2h + pa,
// column X = 2w + pb reads the low-res rows h + pa + rr - 1 and columns w + pb + ss - 1
// (rr, ss in {0, 1}), so the gradient of the 4 phases' 2x2 weights is
//   D[pa pb][co][(rr ss), ci] = sum_{h, w} dy[2h + pa][2w + pb][co] * x[h + pa + rr - 1][w + pb + ss - 1][ci]
// (4/9 of the MACs of the upsampled 3x3; wgrad_reduce_subpix folds the phases back).  A block
// owns 64 co x 64 ci x all 16 (phase, tap) pairs and walks the low-res rows of `spb` consecutive
// (image, 64-column output strip) units.  Step h = output rows 2h, 2h + 1 (one dy group, 2 x 8
// KB) and the low-res x rows h - 1 .. h + 1 (a ring; one new 34-pixel row per step).  The dy
// rows land PHASE-MAJOR in LDS -- LDS row pb * 32 + w holds output pixel 2w + pb (the per-lane
// DMA source chooses the pixel) -- so a phase's A fragment (16 co x 32 pixels) is one
// transposed read pair, like every x fragment (16 ci x 32 low-res pixels at column shift
// pb + ss).  Wave (pa, pb, rr) = wave bits (0, 1, 2): 4 co tiles x 2 ss x 4 ci tiles = 32
// accumulators, 4 A + 8 B fragments per 32 MFMAs.  Output: the sub-pixel slab layout of
// conv_wgrad_v2 <SUB> ([phase][split][co][(rr * 2 + ss) * Cin + ci]) and the per-phase bias slab
// (dy sums by an all-ones operand, the rr = 0 waves of ci tile 0).
// ----------------------------------------------------------------------------------------
struct UpWgArgs {
  const void* x;
  const void* dy;
  float* slab;
  float* bslab;
  int Hin, Win, Cout, Cin, ldd;
  int nct, nci, units, spb, nsplit;     // units = images x output strips; spb units per block
  unsigned xbytes, dybytes;
};

template <int AHEAD>
__global__ void __launch_bounds__(512, 1)
conv3_up_wgrad(UpWgArgs a) {
  // a step = 2 low-res rows (4 dy rows): 64 MFMAs per wave between barriers (one low-res row per
  // step measured 170 us per UpBlock2D conv at B = 32: the per-step barrier, waits and DMA issue
  // were not amortised over 32 MFMAs)
  constexpr int RPS = 2;
  constexpr int BC = 64, NSD = AHEAD + 1, NSX = (AHEAD + 1) * RPS + 2;
  constexpr int DYR = 64 * BC * 2, DYB = 2 * RPS * DYR; // one dy row 8 KB (8 pieces), a group 32 KB
  constexpr int XQ = 5, XB = XQ * 1024;               // x row: 34 px x 128 B = 4352 B -> 5 pieces
  constexpr int NDY = 16 * RPS, NPC = NDY + XQ * RPS; // pieces per group: dy rows, then x rows
  __shared__ __attribute__((aligned(1024))) char smem[NSD * DYB + NSX * XB];
  char* const dyr = smem;
  char* const xr_ = smem + NSD * DYB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int pa = wave & 1, pb = (wave >> 1) & 1, rr = wave >> 2;
  const int li = lane & 15, g = lane >> 4;
  // XCD-aware order: the nct x nci tiles of one split (the same dy and x rows) are consecutive
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int ntile = a.nct * a.nci;
  const int tile = blk % ntile, tc = tile % a.nct, tci = tile / a.nct;
  const int split = blk / ntile;
  const int co0 = tc * BC, ci0 = tci * 64;
  const int Wo = 2 * a.Win, strips = Wo >> 6;
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dy), 0, (int)a.dybytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);

  // this wave's pieces of a group: piece `wave` of each of the 2 RPS dy rows (one lane offset
  // for all of them: the lane's source pixel / channel within the strip row), and x pieces
  // xq = wave (+ 8 for waves 0, 1) of the group's RPS x rows (row xq / XQ, piece xq % XQ).  Few
  // wave-uniform values: per-piece conditions and offsets kept in SGPRs spilled 169 of them
  static_assert(NDY == 8 * 2 * RPS && XQ * RPS <= 16, "piece assignment");
  constexpr int NXP = XQ * RPS;
  const int nxw = (NXP - wave + 7) / 8;               // x pieces of this wave (1 or 2)
  const int npw = 2 * RPS + nxw;
  unsigned dyoff;
  {
    const int o = wave * 1024 + lane * 16;
    const int rho = o >> 7, b = o & 127;
    const int co = (((b >> 5) ^ tswz<BC>(rho)) << 4) | (((b >> 4) & 1) << 3);
    const int px = 2 * (rho & 31) + (rho >> 5);       // phase-major rows
    dyoff = (unsigned)((px * a.ldd + co0 + co) * 2);
  }
  int xrho[2], xci[2];
#pragma unroll
  for (int m = 0; m < 2; ++m) {
    const int xq = wave + 8 * m;
    const int o = (xq % XQ) * 1024 + lane * 16;
    const int rho = o >> 7, b = o & 127;
    xci[m] = ci0 + ((((b >> 5) ^ tswz<64>(rho)) << 4) | (((b >> 4) & 1) << 3));
    xrho[m] = rho;                                    // < 34: a pixel of the row
  }

  // lane constants of the transposed reads (rows: the phase's 32 pixels; x rows shifted by
  // pb + ss), as conv3_halo_wgrad2's lcd / lcx
  unsigned lcd[4][2], lcx[2][4][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rl = 8 * g + 4 * h + (li >> 2);
#pragma unroll
    for (int q = 0; q < 4; ++q) lcd[q][h] = (unsigned)timg_off<BC>(pb * 32 + rl, q * 16 + 4 * (li & 3));
#pragma unroll
    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
      for (int u = 0; u < 4; ++u) lcx[ss][u][h] = (unsigned)timg_off<64>(pb + ss + rl, u * 16 + 4 * (li & 3));
  }
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  auto frag2 = [](const char* base, unsigned l0, unsigned l1) {
    FV_LDS char* lb = (FV_LDS char*)(base);
    const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + l0));
    const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + l1));
    const s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  f32x4 acc[4][2][4];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int ss = 0; ss < 2; ++ss)
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[q][ss][u] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[4];
#pragma unroll
  for (int q = 0; q < 4; ++q) accb[q] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.bslab && tci == 0 && rr == 0;
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;

  const int u0 = split * a.spb, u1 = min(a.units, u0 + a.spb);
  const int nstep = a.Hin / RPS;
  for (int un = u0; un < u1; ++un) {
    const int n = un / strips, w0 = (un % strips) * 64, wl0 = w0 >> 1;
    if (un > u0) __syncthreads();                    // the previous unit's last reads of the rings
    // per unit: the x pieces' source offsets with the strip's column validity (0x80000000 =
    // zero fill: halo columns outside the image, LDS rows past the 34 pixels)
    unsigned xv[2];
#pragma unroll
    for (int m = 0; m < 2; ++m) {
      const int col = wl0 - 1 + xrho[m];
      xv[m] = (xrho[m] < 34 && col >= 0 && col < a.Win) ? (unsigned)((col * a.Cin + xci[m]) * 2) : 0x80000000u;
    }
    // x row y (low-res; -1 and Hin are the zero padding) -> ring slot (y + 1) % NSX
    auto issue_x = [&](int y, int m) {
      const int xq = wave + 8 * m;
      const bool rok = y >= 0 && y < a.Hin;
      dma16s(xr, sbase + NSD * DYB + ((y + 1) % NSX) * XB + (xq % XQ) * 1024, rok ? xv[m] : 0x80000000u,
             rok ? (unsigned)((n * a.Hin + y) * a.Win) * (unsigned)a.Cin * 2u : 0u);
    };
    // group i: dy rows 2 RPS i .. + 2 RPS - 1, x rows RPS i + 1 .. RPS i + RPS
    auto issue_group = [&](int i) {
      const unsigned rb = (unsigned)(((n * 2 * a.Hin + 2 * RPS * i) * Wo + w0) * a.ldd) * 2u;
      const unsigned rs = (unsigned)(Wo * a.ldd) * 2u;
#pragma unroll
      for (int k = 0; k < 2 * RPS; ++k)
        dma16s(dr, sbase + (i % NSD) * DYB + k * DYR + wave * 1024, dyoff, rb + k * rs);
#pragma unroll
      for (int m = 0; m < 2; ++m)
        if (m < nxw) issue_x(RPS * i + 1 + (wave + 8 * m) / XQ, m);
    };
    // prologue: x rows -1 .. RPS - 2 = "group -1"'s x rows
#pragma unroll
    for (int m = 0; m < 2; ++m)
      if (m < nxw) issue_x(1 - RPS + (wave + 8 * m) / XQ, m);
#pragma unroll
    for (int i = 0; i < AHEAD; ++i)
      if (i < nstep) issue_group(i);

    for (int i = 0; i < nstep; ++i) {
      // group i landed; the younger groups issued so far (up to AHEAD - 1) may stay in flight
      const int younger = min(AHEAD - 1, nstep - 1 - i);
      wait_vm_dyn(younger * npw);
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      if (i + AHEAD < nstep) issue_group(i + AHEAD);
#pragma unroll
      for (int hh = 0; hh < RPS; ++hh) {
        const int h = RPS * i + hh;
        const char* dys = dyr + (i % NSD) * DYB + (2 * hh + pa) * DYR;   // dy row 2h + pa
        const char* xs = xr_ + ((h + pa + rr) % NSX) * XB;              // low-res row h + pa + rr - 1
        bf16x8 af[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) af[q] = frag2(dys, lcd[q][0], lcd[q][1]);
        bf16x8 bcur = frag2(xs, lcx[0][0][0], lcx[0][0][1]);
#pragma unroll
        for (int t = 0; t < 8; ++t) {
          const int ss = t >> 2, u = t & 3;
          bf16x8 bnext = bcur;
          if (t + 1 < 8) bnext = frag2(xs, lcx[(t + 1) >> 2][(t + 1) & 3][0], lcx[(t + 1) >> 2][(t + 1) & 3][1]);
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q][ss][u] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[q], bcur, acc[q][ss][u], 0, 0, 0);
          bcur = bnext;
        }
        if (do_bias) {
#pragma unroll
          for (int q = 0; q < 4; ++q) accb[q] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[q], ones, accb[q], 0, 0, 0);
        }
      }
    }
  }
  // slab[(phase * nsplit + split)][co][(rr * 2 + ss) * Cin + ci]: lane holds D[co = 4g + jj][ci = li]
  const int ph = pa * 2 + pb;
  const long KW = 4L * a.Cin;
  float* sl = a.slab + (long)(ph * a.nsplit + split) * a.Cout * KW;
#pragma unroll
  for (int ss = 0; ss < 2; ++ss)
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int kcol = (rr * 2 + ss) * a.Cin + ci0 + u * 16 + li;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) sl[(long)(co0 + q * 16 + 4 * g + jj) * KW + kcol] = acc[q][ss][u][jj];
    }
  if (do_bias && li == 0) {
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int jj = 0; jj < 4; ++jj) a.bslab[(long)(ph * a.nsplit + split) * a.Cout + co0 + q * 16 + 4 * g + jj] = accb[q][jj];
  }
}

// ----------------------------------------------------------------------------------------
// Weight gradient of the 7x7 64 -> <= 4 channel conv (Generator.out_conv), "row taps in N":
//   D[(s, ci)][(r, co)] = sum_{x row h, column w} x[h][w + s - 3][ci] * dy[h - r + 3][w][co]
//                      = dW[co][ci][r][s]
// M = 7 column taps x 64 ci = 448 (28 m-tiles), N = 7 row taps x 4 co = 28 of 32 (2 n-tiles),
// K = x pixels: 3.5x fewer MFMAs than M = 3136, N = 3 -> 16.  A block walks the x rows of a
// 64-column strip segment: per row the x row (70 columns incl. the column halo) lands in LDS
// by DMA (double buffered) and the dy row 3 below it is transposed into a ring of 8
// channel-major dy rows, from which a B fragment (8 consecutive columns of one (r, co)) is a
// single ds_read_b128; A fragments are transposed reads (pixels are the MFMA K) of the x row.
// Output: per-block fp32 slabs [block][32][448] (n = r*4 + co, m = s*64 + ci) + bias sums.
// ----------------------------------------------------------------------------------------
struct W7Args {
  const void* x;
  const void* dy;
  float* slab;
  float* bslab;
  int H, W, ldd, cout, seg_rows, nseg;
  unsigned xbytes, dybytes;
};

__global__ void __launch_bounds__(512, 2)
conv7_n3_wgrad(W7Args a) {
  constexpr int XROW = 9 * 1024;                            // 70 px x 128 B, padded to whole pieces
  constexpr int XQ = 70 * 128 / 1024 + 1;                    // 9 pieces (the last one partly past 70 px)
  __shared__ __attribute__((aligned(1024))) char smem[2 * XROW + 2 * 1024 + 8 * 512];
  char* xb = smem;                                           // [2][70 px][64 ci] (timg_off<64> layout)
  char* dys = smem + 2 * XROW;                               // [2][64 px][8 ch] as stored in dy
  bf16* dyT = reinterpret_cast<bf16*>(smem + 2 * XROW + 2 * 1024);   // [8 rows][4 co][64 w]
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int li = lane & 15, g = lane >> 4;
  const int strips = a.W / 64;
  const int blk = blockIdx.x;
  const int seg = blk % a.nseg, strip = (blk / a.nseg) % strips, n = blk / (a.nseg * strips);
  const int w0 = strip * 64;
  const int hb = seg * a.seg_rows, he = min(a.H, hb + a.seg_rows);
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dy), 0, (int)a.dybytes, 0x00020000);

  // x row h -> xb[buf] (pixel p = column w0 - 3 + p; 32-B blocks XOR-swizzled, timg_off<64>)
  auto issue_x = [&](int h, int buf) {
    for (int q = wave; q < XQ; q += 8) {
      const int o = q * 1024 + lane * 16;
      const int p = o >> 7, b = o & 127;
      const int ci = ((((b >> 5) ^ tswz<64>(p)) << 4) | (((b >> 4) & 1) << 3));
      const int ww = w0 - 3 + p;
      const bool ok = p < 70 && h >= 0 && h < a.H && ww >= 0 && ww < a.W;
      dma16(xr, xb + buf * XROW + q * 1024,
            ok ? (unsigned)((((n * a.H + h) * a.W + ww) * 64 + ci) * 2) : 0x80000000u);
    }
  };
  // dy row y (64 px x ldd = 8 channels = 1 KB) -> dys[buf], one piece by wave 0
  auto issue_dy = [&](int y, int buf) {
    if (wave == 0) {
      const bool ok = y >= 0 && y < a.H;
      dma16(dr, dys + buf * 1024, ok ? (unsigned)((((n * a.H + y) * a.W + w0) * 8) * 2 + lane * 16) : 0x80000000u);
    }
  };
  // dys[buf] -> dyT[y & 7] (channel-major; zero rows outside the image / channels >= cout)
  auto transpose_dy = [&](int y, int buf) {
    if (tid < 256) {
      const int w = tid & 63, co = tid >> 6;
      const bf16 v = (y >= 0 && y < a.H && co < a.cout) ? reinterpret_cast<const bf16*>(dys + buf * 1024)[w * 8 + co]
                                                          : (bf16)0.f;
      dyT[((y & 7) * 4 + co) * 64 + w] = v;
    }
  };

  // prologue: dy rows hb-3 .. hb+2 straight into the ring (plain loads), first x / dy DMAs
  for (int e = tid; e < 6 * 256; e += 512) {
    const int y = hb - 3 + e / 256, w = e & 63, co = (e >> 6) & 3;
    bf16 v = (bf16)0.f;
    if (y >= 0 && y < a.H && co < a.cout)
      v = reinterpret_cast<const bf16*>(a.dy)[((long)(n * a.H + y) * a.W + w0 + w) * 8 + co];
    dyT[((y & 7) * 4 + co) * 64 + w] = v;
  }
  issue_x(hb, 0);
  issue_dy(hb + 3, 0);

  // this wave's m-tiles: w, w + 8, w + 16, w + 24 (< 28), each with both n-tiles
  const int nmt = wave < 4 ? 4 : 3;
  f32x4 acc[4][2];
#pragma unroll
  for (int i = 0; i < 4; ++i) acc[i][0] = acc[i][1] = f32x4{0.f, 0.f, 0.f, 0.f};
  float bsum = 0.f;                                          // bias gradient: this thread's (w, co)

  for (int h = hb; h < he; ++h) {
    const int buf = (h - hb) & 1;
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();                                         // x row h, dy row h+3 landed; step h-1 done
    transpose_dy(h + 3, buf);
    if (h + 1 < he) {
      issue_x(h + 1, buf ^ 1);
      issue_dy(h + 4, buf ^ 1);
    }
    __syncthreads();                                         // dy row h+3 visible in the ring
    if (tid < 256) {
      const int w = tid & 63, co = tid >> 6;
      bsum += (float)dyT[((h & 7) * 4 + co) * 64 + w];
    }
    const char* xbuf = xb + buf * XROW;
#pragma unroll
    for (int kk = 0; kk < 2; ++kk) {
      bf16x8 bfr[2];
#pragma unroll
      for (int t = 0; t < 2; ++t) {
        const int nn = t * 16 + li, r = nn >> 2, co = nn & 3;
        const int y = h - r + 3;
        bf16x8 v = *reinterpret_cast<const bf16x8*>(dyT + ((y & 7) * 4 + co) * 64 + kk * 32 + g * 8);
        if (r > 6) v = bf16x8{};
        bfr[t] = v;
      }
#pragma unroll
      for (int i = 0; i < 4; ++i) {
        if (i < nmt) {
          const int mt = wave + 8 * i, s7 = mt >> 2, cb = (mt & 3) * 16;
          const bf16x8 afr = tfrag<64>(xbuf, kk * 32 + s7, cb, lane);
          acc[i][0] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[0], acc[i][0], 0, 0, 0);
          acc[i][1] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr, bfr[1], acc[i][1], 0, 0, 0);
        }
      }
    }
  }
  // slab[blk][n][m]: lane holds D[m = mt*16 + 4g + j][n = t*16 + li]
  float* sl = a.slab + (long)blk * 32 * 448;
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    if (i < nmt) {
      const int mt = wave + 8 * i;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int j = 0; j < 4; ++j) sl[(t * 16 + li) * 448 + mt * 16 + 4 * g + j] = acc[i][t][j];
    }
  }
  // bias: sum over the 64 columns of each co (waves 0..3 hold co = wave)
  if (a.bslab && tid < 256) {
    const float t = wave_sum(bsum);
    if (lane == 0) a.bslab[blk * 4 + wave] = t;
  }
}

// slabs [nblk][32][448] + [nblk][4] -> dW[co][64][7][7], db[co] in two deterministic passes.
// Pass 1: block (column chunk, group g) sums the slab rows [g*rpg, (g+1)*rpg) of 64 columns
// (4 waves x rows strided by 4, 4 loads in flight per lane) and stores the partial in place
// over row g*rpg.  Pass 2 sums the G partials in order.  Column e < 12544 is slab element
// (n = e / 448, m = e % 448); e in [12544, 12548) is bias co = e - 12544.
constexpr int W7_COLS = 28 * 448;
__device__ __forceinline__ float* w7_elem(float* slab, float* bslab, int b, int e) {
  return e < W7_COLS ? slab + (long)b * 32 * 448 + e : bslab + b * 4 + (e - W7_COLS);
}

__global__ void __launch_bounds__(256)
w7_reduce1_kernel(float* slab, float* bslab, int nblk, int rpg, int ncol) {
  const int e = blockIdx.x * 64 + (threadIdx.x & 63), sg = threadIdx.x >> 6;
  const int b0 = blockIdx.y * rpg, b1 = min(nblk, b0 + rpg);
  __shared__ float red[4][64];
  float acc[4] = {0.f, 0.f, 0.f, 0.f};
  if (e < ncol) {
    int b = b0 + sg;
    for (; b + 12 < b1; b += 16) {
#pragma unroll
      for (int u = 0; u < 4; ++u) acc[u] += *w7_elem(slab, bslab, b + 4 * u, e);
    }
    for (; b < b1; b += 4) acc[0] += *w7_elem(slab, bslab, b, e);
  }
  red[sg][threadIdx.x & 63] = (acc[0] + acc[1]) + (acc[2] + acc[3]);
  __syncthreads();
  if (sg == 0 && e < ncol && b0 < b1)
    *w7_elem(slab, bslab, b0, e) = (red[0][threadIdx.x] + red[1][threadIdx.x]) + (red[2][threadIdx.x] + red[3][threadIdx.x]);
}

__global__ void w7_reduce2_kernel(float* slab, float* bslab, int nblk, int rpg, int cout, float* dw, float* db) {
  const int e = blockIdx.x * blockDim.x + threadIdx.x;
  if (e >= W7_COLS + (db ? cout : 0)) return;
  const int nn = e / 448, co = nn & 3;
  if (e < W7_COLS && co >= cout) return;
  float v = 0.f;
  for (int b = 0; b < nblk; b += rpg) v += *w7_elem(slab, bslab, b, e);
  if (e < W7_COLS) {
    const int r = nn >> 2, m = e - nn * 448, s7 = m >> 6, ci = m & 63;
    dw[((co * 64 + ci) * 7 + r) * 7 + s7] = v;
  } else {
    db[e - W7_COLS] = v;
  }
}

// ----------------------------------------------------------------------------------------
// Halo-tiled 7x7 weight gradient (bf16): Generator.out_conv 64->3 and AFE.in_conv 3->64.
//   dW[co][k = (tap, ci)] = sum_p dy[p][co] * x[p + off(tap)][ci]      (M = k, N = co, K = p)
// Persistent blocks (one per CU) walk TR x 64 pixel tiles; per tile the input halo and the
// dy tile land in LDS by DMA (double-buffered: tile t+1 streams in while t is computed),
// and every tap's A fragment is a transposed read (ds_read_b64_tr_b16) of the halo at the
// tap's shift -- the input is read from HBM ~once instead of 49x.  Accumulators stay in
// registers across tiles; one fp32 slab per block, reduced by wgrad_reduce_kernel.  The
// bias gradient uses the all-ones A operand trick (wave 0).
// Wave w owns n-tile (w % NT) and m-tiles w/NT, w/NT + 8/NT, ...  (NT = co tiles).
// ----------------------------------------------------------------------------------------
struct HaloWgArgs {
  const void* x;
  const void* dy;
  float* slab;
  float* bslab;
  int H, W, ldd, K, KW, CW, ntiles, cout;
  unsigned xbytes, dybytes;
};

// PK (AFE.in_conv, <= 4 valid input channels of the 8 staged per pixel): k packed as
// k = r * 32 + s * 4 + ci (s = 7 a padding column, ci = 3 the zero channel), the weight layout
// conv7c4_fwd's forward reads -- 14 m-tiles instead of 25 (49 taps x 8 padded channels): a
// lane's 4 k are ci 0..3 of one tap = the first 8 B of the halo pixel at that tap's shift.
// The slab rows are these k (KW = 224); wgrad_reduce_kernel maps them back (KSL = 8).
template <int KS, int CIN, int NT, int TR, bool PK = false>
__global__ void __launch_bounds__(512, 2)
conv_halo_wgrad(HaloWgArgs a) {
  static_assert(!PK || (CIN == 8 && KS == 7), "packed 7x7 weight gradient: 8 staged channels");
  constexpr int PAD = KS / 2, TW = 64;
  constexpr int HR = TR + KS - 1, HW = TW + KS - 1;
  constexpr int CPP = CIN / 8;
  constexpr int HCH = HR * HW * CPP;
  constexpr int HQ = (HCH + 63) / 64;
  constexpr int LDD = NT == 1 ? 8 : NT * 16;       // dy channels staged per pixel
  constexpr int DCH = TR * TW * LDD / 8;
  constexpr int DQ = (DCH + 63) / 64;
  constexpr int HB = HQ * 1024, DB = DQ * 1024, BUF = HB + DB;
  constexpr int KT = PK ? KS * 32 : KS * KS * CIN;  // valid k
  constexpr int MTT = (KT + 15) / 16;               // m-tiles (16 k rows)
  // every wave owns m-tiles {wave, wave + 8, ...} and ALL NT n-tiles: the A fragment of an
  // m-tile (two transposed 8-B halo reads) feeds NT MFMAs.  (One n-tile per wave, as before,
  // paid two LDS reads per MFMA: LDS-bound at 21 % MFMA busy on AFE.in_conv, NT = 4.)
  constexpr int RMW = (MTT + 7) / 8;                // m-tiles per wave (max)
  constexpr int NKG = TR * TW / 32;                 // 32-pixel k-groups per tile
  __shared__ __attribute__((aligned(1024))) char smem[2 * BUF];

  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int mw = wave;
  const int li = lane & 15, g = lane >> 4, q4 = li >> 2, pp = li & 3;
  const int tiles_w = a.W / TW, tiles_h = a.H / TR;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.dy), 0, (int)a.dybytes, 0x00020000);

  auto issue = [&](int tile, int buf) {
    const int n = tile / (tiles_h * tiles_w);
    const int rem = tile - n * tiles_h * tiles_w;
    const int h0 = (rem / tiles_w) * TR, w0 = (rem % tiles_w) * TW;
    char* halo = smem + buf * BUF;
    char* dys = halo + HB;
    for (int q = wave; q < HQ; q += 8) {
      const int L = q * 64 + lane;
      const int hp = L / CPP, ch = L - (L / CPP) * CPP;
      const int hr = hp / HW, hc = hp - (hp / HW) * HW;
      const int hh = h0 + hr - PAD, ww = w0 + hc - PAD;
      const int sc = ch ^ (hp & (CPP - 1));
      const bool ok = L < HCH && hh >= 0 && hh < a.H && ww >= 0 && ww < a.W;
      const unsigned off = ok ? (unsigned)((((n * a.H + hh) * a.W + ww) * CIN + sc * 8) * 2) : 0x80000000u;
      dma16(xr, halo + q * 1024, off);
    }
    for (int q = wave; q < DQ; q += 8) {
      const int L = q * 64 + lane;
      constexpr int CPR = LDD / 8;
      const int row = L / CPR, dch = L - (L / CPR) * CPR;
      const int sc = CPR >= 4 ? ((((dch >> 1) ^ tswz<LDD>(row)) << 1) | (dch & 1)) : dch;
      const int p = (n * a.H + h0 + row / TW) * a.W + w0 + (row % TW);
      const bool ok = L < DCH && sc * 8 < a.ldd;
      const unsigned off = ok ? (unsigned)((p * a.ldd + sc * 8) * 2) : 0x80000000u;
      dma16(dr, dys + q * 1024, off);
    }
  };

  // this lane's constant part of each A fragment: (tap offset, byte offset in the pixel)
  int aoff[RMW], akx[RMW];
  bool aok[RMW];
#pragma unroll
  for (int j = 0; j < RMW; ++j) {
    const int mt = mw + j * 8;
    const int k = mt * 16 + 4 * pp;                 // first of this lane's 4 k (same tap, same chunk)
    aok[j] = mt < MTT;                              // wave-uniform (transposed reads need EXEC = all)
    if constexpr (PK) {
      // s = 7 reads one column past the tap window (the next halo row's first pixel, or the
      // dy image after the last row): finite junk in rows the reduce never maps
      aoff[j] = k < KT ? (k >> 5) * HW + ((k >> 2) & 7) : 0;
      akx[j] = 0;
    } else {
      const int tap = k / CIN, ci = k - (k / CIN) * CIN;
      const int r = tap / KS, s = tap - (tap / KS) * KS;
      aoff[j] = k < KT ? r * HW + s : 0;            // k >= K rows: finite junk, never stored
      akx[j] = k < KT ? ci : 0;
    }
  }
  f32x4 acc[RMW][NT];
#pragma unroll
  for (int j = 0; j < RMW; ++j)
#pragma unroll
    for (int n = 0; n < NT; ++n) acc[j][n] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[NT];
#pragma unroll
  for (int n = 0; n < NT; ++n) accb[n] = f32x4{0.f, 0.f, 0.f, 0.f};
  const bool do_bias = a.bslab && wave == 7;        // a wave with the fewest m-tiles
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;

  // fragments of k-group kg (B: dy[32 px][16 co] of every n-tile; A: the halo at each m-tile's
  // tap shift), all reads issued together before the k-group's MFMAs (one m-tile's 2 reads
  // right before its 4 MFMAs left the LDS latency exposed: AFE.in_conv 140.7 -> 131.4 us; the
  // k-groups double-buffered as well spill at 256 registers: 145.7)
  auto load_kg = [&](const char* halo, int kg, bf16x8 (&bfr)[NT], bf16x8 (&afr)[RMW]) {
    const char* dys = halo + HB;
    FV_LDS char* hl = (FV_LDS char*)(halo);
#pragma unroll
    for (int n = 0; n < NT; ++n) bfr[n] = tfrag<LDD>(dys, kg * 32, n * 16, lane);   // co >= LDD lanes: ignored
    // pixel rows 8g+q4 and 8g+4+q4 of this k-group -> halo pixel at tap (0,0)
    const int p0 = kg * 32 + 8 * g + q4, p1 = p0 + 4;
    const int hb0 = (p0 / TW) * HW + (p0 % TW), hb1 = (p1 / TW) * HW + (p1 % TW);
#pragma unroll
    for (int j = 0; j < RMW; ++j) {
      afr[j] = bf16x8{};
      if (aok[j]) {
        const int ha = hb0 + aoff[j], hb = hb1 + aoff[j];
        const int ca = ((akx[j] >> 3) ^ (ha & (CPP - 1))) * 16 + (akx[j] & 7) * 2;
        const int cb = ((akx[j] >> 3) ^ (hb & (CPP - 1))) * 16 + (akx[j] & 7) * 2;
        const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(hl + ha * CIN * 2 + ca));
        const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(hl + hb * CIN * 2 + cb));
        typedef short s16x8 __attribute__((ext_vector_type(8)));
        const s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
        afr[j] = __builtin_bit_cast(bf16x8, v);
      }
    }
  };
  auto mfma_kg = [&](const bf16x8 (&bfr)[NT], const bf16x8 (&afr)[RMW]) {
#pragma unroll
    for (int j = 0; j < RMW; ++j)
#pragma unroll
      for (int n = 0; n < NT; ++n) acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(afr[j], bfr[n], acc[j][n], 0, 0, 0);
    if (do_bias) {
#pragma unroll
      for (int n = 0; n < NT; ++n) accb[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bfr[n], accb[n], 0, 0, 0);
    }
  };
  auto compute = [&](int buf) {
    const char* halo = smem + buf * BUF;
    if constexpr (RMW * NT <= 16) {
      for (int kg = 0; kg < NKG; ++kg) {
        bf16x8 b0[NT], a0[RMW];
        load_kg(halo, kg, b0, a0);
        mfma_kg(b0, a0);
      }
    } else {
      // many m-tiles per wave (64-channel input): each A fragment read right before its MFMAs
      const char* dys = halo + HB;
      FV_LDS char* hl = (FV_LDS char*)(halo);
      for (int kg = 0; kg < NKG; ++kg) {
        bf16x8 bfr[NT];
#pragma unroll
        for (int n = 0; n < NT; ++n) bfr[n] = tfrag<LDD>(dys, kg * 32, n * 16, lane);
        const int p0 = kg * 32 + 8 * g + q4, p1 = p0 + 4;
        const int hb0 = (p0 / TW) * HW + (p0 % TW), hb1 = (p1 / TW) * HW + (p1 % TW);
#pragma unroll
        for (int j = 0; j < RMW; ++j) {
          bf16x8 af = bf16x8{};
          if (aok[j]) {
            const int ha = hb0 + aoff[j], hb = hb1 + aoff[j];
            const int ca = ((akx[j] >> 3) ^ (ha & (CPP - 1))) * 16 + (akx[j] & 7) * 2;
            const int cb = ((akx[j] >> 3) ^ (hb & (CPP - 1))) * 16 + (akx[j] & 7) * 2;
            const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(hl + ha * CIN * 2 + ca));
            const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(hl + hb * CIN * 2 + cb));
            typedef short s16x8 __attribute__((ext_vector_type(8)));
            const s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
            af = __builtin_bit_cast(bf16x8, v);
          }
#pragma unroll
          for (int n = 0; n < NT; ++n) acc[j][n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af, bfr[n], acc[j][n], 0, 0, 0);
        }
        if (do_bias) {
#pragma unroll
          for (int n = 0; n < NT; ++n) accb[n] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ones, bfr[n], accb[n], 0, 0, 0);
        }
      }
    }
  };

  int tile = blockIdx.x;
  if (tile < a.ntiles) issue(tile, 0);
  for (int it = 0; tile < a.ntiles; ++it, tile += gridDim.x) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    if (tile + (int)gridDim.x < a.ntiles) issue(tile + gridDim.x, (it + 1) & 1);
    compute(it & 1);
  }

  // D[k][co]: lane holds k = mt*16 + 4*(lane>>4) + i for co = nt*16 + (lane & 15)
  float* slab = a.slab + (long)blockIdx.x * a.CW * a.KW;
#pragma unroll
  for (int n = 0; n < NT; ++n) {
    const int co = n * 16 + li;
    if (co < a.cout) {
#pragma unroll
      for (int j = 0; j < RMW; ++j) {
        const int mt = mw + j * 8;
        if (mt < MTT)
          *reinterpret_cast<float4*>(slab + (long)co * a.KW + mt * 16 + g * 4) =
              make_float4(acc[j][n][0], acc[j][n][1], acc[j][n][2], acc[j][n][3]);
      }
      if (do_bias && g == 0) a.bslab[(long)blockIdx.x * a.CW + co] = accb[n][0];
    }
  }
}

// ----------------------------------------------------------------------------------------
// weight re-layout (+ 1/sigma) and slab reduction
// ----------------------------------------------------------------------------------------
// smaj 2: the packed 7x7 layout of conv7c4_fwd ([row][224], 2 taps x 4 channels per 16 B).
// smaj 1 (the layout conv3_halo_fwd3 reads, h3s_layout): stage-major [u = c * 9 + tap][row][32]
// with c the 32-channel chunk, so every 16-row DMA piece of a weight stage is one contiguous
// 1 KB (8 whole 128-B lines) instead of 16 row segments of 64 B.  Requires KS == 3,
// Kpad == 9 * Cin and Cin % 32 == 0.
template <typename T>
__device__ __forceinline__ void weight_prep_body(const float* __restrict__ wp, const float* sigma, T* wk, int rows,
                                                 int Kpad, int cout, int cin_valid, int lgCin, int KS, int K,
                                                 int transposed, int bid, int nblk, int smaj = 0) {
  // 32-bit index math (a weight image is < 2^31 elements; the 64-bit divisions per element
  // dominated the batched launch)
  const int total = rows * Kpad;
  const float inv = sigma ? 1.f / sigma[0] : 1.f;
  for (int e = bid * (int)blockDim.x + threadIdx.x; e < total; e += nblk * (int)blockDim.x) {
    int row, k;
    bool kin;
    int tap, c;
    if (smaj == 2) {            // conv7c4_fwd: [row][224], k = r * 32 + s * 4 + ci (s = 7: zero)
      row = e / C74_K;
      k = e - row * C74_K;
      const int sk = (k >> 2) & 7;
      kin = sk < 7;
      tap = (k >> 5) * 7 + sk;
      c = k & 3;
    } else {
      if (smaj) {
        const int q = e >> 5, u = q / rows;
        row = q - u * rows;
        const int cc = u / 9, t = u - cc * 9;
        k = (t << lgCin) + cc * 32 + (e & 31);
      } else {
        row = e / Kpad;
        k = e - row * Kpad;
      }
      kin = k < K;
      tap = k >> lgCin;
      c = k & ((1 << lgCin) - 1);
    }
    float v = 0.f;
    if (kin) {
      const int r = tap / KS, s = tap - (tap / KS) * KS;
      if (!transposed) {        // wk[co][(r,s,ci)] = W[co][ci][r][s]
        if (row < cout && c < cin_valid) v = wp[(((long)row * cin_valid + c) * KS + r) * KS + s];
      } else {                  // wt[ci][(r',s',co)] = W[co][ci][KS-1-r'][KS-1-s']
        if (row < cin_valid && c < cout)
          v = wp[(((long)c * cin_valid + row) * KS + (KS - 1 - r)) * KS + (KS - 1 - s)];
      }
    }
    wk[e] = Elt<T>::from_f(v * inv);
  }
}

template <typename T>
__global__ void weight_prep_kernel(const float* __restrict__ wp, const float* sigma, T* wk,
                                   int rows, int Kpad, int cout, int cin_valid, int lgCin, int KS,
                                   int K, int transposed, int smaj) {
  weight_prep_body<T>(wp, sigma, wk, rows, Kpad, cout, cin_valid, lgCin, KS, K, transposed, blockIdx.x, gridDim.x,
                      smaj);
}

// both layouts in one launch: blocks [0, nb1) write wk, the rest wt
struct WPrepJob { void* out; int rows, Kpad, lgCin, K, transposed, nb, smaj; };
template <typename T>
__global__ void weight_prep2_kernel(const float* __restrict__ wp, const float* sigma, int cout, int cin_valid, int KS,
                                    WPrepJob j0, WPrepJob j1) {
  const bool second = (int)blockIdx.x >= j0.nb;
  const WPrepJob& j = second ? j1 : j0;
  weight_prep_body<T>(wp, sigma, (T*)j.out, j.rows, j.Kpad, cout, cin_valid, j.lgCin, KS, j.K, j.transposed,
                      second ? blockIdx.x - j0.nb : blockIdx.x, j.nb, j.smaj);
}

// one launch for the generic weight layouts of many convs (fv_conv_weight_prep_multi): job j
// owns blocks [blk0, blk0 + nb); at most 2 * FV_WPREP_MAX jobs, passed by value
struct WPrepMJob {
  const float* w;
  const float* sigma;
  void* out;
  int rows, Kpad, lgCin, K, transposed, nb, cout, cin_valid, KS, blk0, smaj;
};
struct WPrepMulti {
  int n;
  WPrepMJob j[2 * FV_WPREP_MAX];
};
// grid (max nb, jobs): blockIdx.y selects the job directly (a per-block search over the job
// list in kernel-argument memory cost more than the launches it replaced)
template <typename T>
__global__ void weight_prep_multi_kernel(WPrepMulti m) {
  const WPrepMJob& j = m.j[blockIdx.y];
  if ((int)blockIdx.x >= j.nb) return;
  weight_prep_body<T>(j.w, j.sigma, (T*)j.out, j.rows, j.Kpad, j.cout, j.cin_valid, j.lgCin, j.KS, j.K, j.transposed,
                      blockIdx.x, j.nb, j.smaj);
}

// sub-pixel phase weights of an upsample + 3x3 conv: for phase (pa, pb) the 2x2 tap (r', s')
// sums the 3x3 taps that land on the same low-res input pixel (rows r in [lo, hi] with
// lo = r' ? 1 + pa : 0, hi = r' ? 2 : pa; columns alike).  wk [4][rows][Kpad], k = (r'*2+s')*cin + ci.
template <typename T>
__global__ void weight_prep_subpix_kernel(const float* __restrict__ wp, const float* sigma, T* wk, int rows, int Kpad,
                                          int cout, int cin_valid, int lgCin) {
  const long per = (long)rows * Kpad, total = 4 * per;
  const float inv = sigma ? 1.f / sigma[0] : 1.f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int ph = (int)(e / per);
    const long e2 = e - ph * per;
    const int row = (int)(e2 / Kpad), k = (int)(e2 - (long)row * Kpad);
    const int pa = ph >> 1, pb = ph & 1;
    const int tap = k >> lgCin, c = k & ((1 << lgCin) - 1);
    float v = 0.f;
    if (tap < 4 && row < cout && c < cin_valid) {
      const int rr = tap >> 1, ss = tap & 1;
      const int r0 = rr ? 1 + pa : 0, r1 = rr ? 2 : pa;
      const int s0 = ss ? 1 + pb : 0, s1 = ss ? 2 : pb;
      const float* w = wp + ((long)row * cin_valid + c) * 9;
      for (int r = r0; r <= r1; ++r)
        for (int q = s0; q <= s1; ++q) v += w[r * 3 + q];
    }
    wk[e] = Elt<T>::from_f(v * inv);
  }
}

// stride-2 4x4 weights of the low-res data gradient of an upsample + 3x3 conv:
// wt[ci][(tr*4 + tc)*cin_t + co] = sum of W[co][ci][r][s] over r in [max(0, 2-tr), min(2, 3-tr)]
// and s alike (dy row 2u + tr - 1 reaches low-res row u through those taps).
template <typename T>
__global__ void weight_prep_s2_kernel(const float* __restrict__ wp, const float* sigma, T* wt, int rows, int Kpad,
                                      int cout, int cin_valid, int lgCt) {
  const long total = (long)rows * Kpad;
  const float inv = sigma ? 1.f / sigma[0] : 1.f;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < total; e += (long)gridDim.x * blockDim.x) {
    const int row = (int)(e / Kpad), k = (int)(e - (long)row * Kpad);
    const int tap = k >> lgCt, co = k & ((1 << lgCt) - 1);
    float v = 0.f;
    if (tap < 16 && row < cin_valid && co < cout) {
      const int tr = tap >> 2, tc = tap & 3;
      const int r0 = max(0, 2 - tr), r1 = min(2, 3 - tr), s0 = max(0, 2 - tc), s1 = min(2, 3 - tc);
      const float* w = wp + ((long)co * cin_valid + row) * 9;
      for (int r = r0; r <= r1; ++r)
        for (int q = s0; q <= s1; ++q) v += w[r * 3 + q];
    }
    wt[e] = Elt<T>::from_f(v * inv);
  }
}

// Weight images of conv3_halo_fwd3 MODE 1 / 2: unit u = chunk c * 4 + q, a [rows][32] block per
// unit (stage-major, as weight_prep_body smaj 1), q = (q >> 1, q & 1).
//   MODE 1 (sub-pixel forward, wk): rows = 4 cout, row = tn * 256 + phase * 64 + co % 64 for
//     co = tn * 64 + co % 64; element k = input channel c * 32 + k: phase (pa, pb)'s 2x2 tap
//     (rr, ss) = q, the folded 3x3 sum of weight_prep_subpix_kernel.
//   MODE 2 (low-res data gradient, wt): rows = the tile rows (cin of the conv), chunk c = (plane
//     (py, px) = c / cpp, 32 output channels (c % cpp) * 32 + k); q = (a, b) is the stride-2
//     tap (tr, tc) = (2a + 1 - py, 2b + 1 - px) of weight_prep_s2_kernel.
// CONVT: the ConvTranspose2dELR k4 s2 p1 weights w [ci][co][4][4] (x gain (x cinv[co], demod))
// on the same kernels: phase (pa, pb) tap (rr, ss) SELECTS Weff[ci][co][3 - pa - 2 rr][3 - pb - 2 ss]
// (convt_weight_prep_kernel's map), and the stride-2 data-gradient tap (tr, tc) is Weff[ci][co][tr][tc].
template <int MODE, bool CONVT = false>
__global__ void weight_prep_phase_kernel(const float* __restrict__ wp, const float* sigma, bf16* out, int rows,
                                         int units, int cout, int cin_valid, int cpp, const float* cinv = nullptr,
                                         float gain = 1.f) {
  const int total = units * rows * 32;
  const float inv = sigma ? 1.f / sigma[0] : 1.f;
  for (int e = blockIdx.x * (int)blockDim.x + threadIdx.x; e < total; e += gridDim.x * (int)blockDim.x) {
    const int k = e & 31, qe = e >> 5, u = qe / rows, row = qe - u * rows;
    const int c = u >> 2, q = u & 3;
    int co, ci, r0, r1, s0, s1;
    if constexpr (MODE == 1) {
      const int ph = (row >> 6) & 3, pa = ph >> 1, pb = ph & 1, rr = q >> 1, ss = q & 1;
      co = (row >> 8) * 64 + (row & 63);
      ci = c * 32 + k;
      r0 = rr ? 1 + pa : 0; r1 = rr ? 2 : pa;
      s0 = ss ? 1 + pb : 0; s1 = ss ? 2 : pb;
    } else {
      const int pl = c / cpp, tr = 2 * (q >> 1) + 1 - (pl >> 1), tc = 2 * (q & 1) + 1 - (pl & 1);
      co = (c - pl * cpp) * 32 + k;
      ci = row;
      r0 = max(0, 2 - tr); r1 = min(2, 3 - tr);
      s0 = max(0, 2 - tc); s1 = min(2, 3 - tc);
    }
    float v = 0.f;
    if (co < cout && ci < cin_valid) {
      if constexpr (CONVT) {
        int tr, tc;
        if constexpr (MODE == 1) {
          tr = 3 - ((row >> 7) & 1) - 2 * (q >> 1);
          tc = 3 - ((row >> 6) & 1) - 2 * (q & 1);
        } else {
          const int pl = c / cpp;
          tr = 2 * (q >> 1) + 1 - (pl >> 1);
          tc = 2 * (q & 1) + 1 - (pl & 1);
        }
        v = wp[((long)ci * cout + co) * 16 + tr * 4 + tc] * (cinv ? gain * cinv[co] : gain);
      } else {
        const float* w = wp + ((long)co * cin_valid + ci) * 9;
        for (int r = r0; r <= r1; ++r)
          for (int t = s0; t <= s1; ++t) v += w[r * 3 + t];
      }
    }
    out[e] = Elt<bf16>::from_f(CONVT ? v : v * inv);
  }
}

// sub-pixel phase slabs [4][nsplit][CW][KW] (k = (r'*2+s')*cin + ci) -> dW [co][ci][3][3]:
// each 3x3 tap r takes, per phase row pa, the 2x2 tap r' whose folded range holds it
// (pa = 0: r' = r > 0; pa = 1: r' = r == 2), columns alike; + db from the bias slabs.
// One wave per 64 outputs, 4 lanes per output summing interleaved splits.
__global__ void wgrad_reduce_subpix_kernel(const float* __restrict__ slab, const float* __restrict__ bslab, float* dw,
                                           float* db, int nsplit, int CW, int KW, int cout, int cin_valid,
                                           int lgCin, int nb_main) {
  const int sg = threadIdx.x >> 6, l = threadIdx.x & 63;
  __shared__ float red[4][64];
  float g = 0.f;
  long dst = -1;
  const int nterm = 4 * nsplit;
  if ((int)blockIdx.x < nb_main) {
    const long e = (long)blockIdx.x * 64 + l;
    const long tot = (long)cout * cin_valid * 9;
    if (e < tot) {
      dst = e;
      const int rs = (int)(e % 9), ci = (int)((e / 9) % cin_valid), co = (int)(e / (9L * cin_valid));
      const int r = rs / 3, sc = rs % 3;
      for (int t = sg; t < nterm; t += 4) {
        const int ph = t / nsplit, sp = t - ph * nsplit;
        const int pa = ph >> 1, pb = ph & 1;
        const int rr = pa ? (r == 2) : (r > 0), ss = pb ? (sc == 2) : (sc > 0);
        g += slab[((long)(ph * nsplit + sp) * CW + co) * KW + (((rr * 2 + ss) << lgCin) + ci)];
      }
    }
  } else {
    const int co = ((int)blockIdx.x - nb_main) * 64 + l;
    if (co < cout) {
      dst = co;
      for (int t = sg; t < nterm; t += 4) g += bslab[(long)t * CW + co];
    }
  }
  red[sg][l] = g;
  __syncthreads();
  if (sg == 0 && dst >= 0) {
    const float v = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    if ((int)blockIdx.x < nb_main) dw[dst] = v;
    else db[dst] = v;
  }
}

// Sub-pixel slabs of many splits (conv3_up_wgrad: ~one block per CU, 4 x 128 splits at
// 256^2), in two passes instead of the gather above (whose 9 (r, s) neighbours read 4 rows a
// cin apart: 117 us for the two UpBlock2D convs at B = 32):
// pass 1 sums each phase's splits over 64 consecutive slab elements x 4 split lanes (coalesced,
// fixed order) and writes the sum in place into the phase's split-0 row (every element is read
// by its own block only); blocks >= nb_main do the same for the bias slab.
__global__ void subpix_split_sum_kernel(float* __restrict__ slab, float* __restrict__ bslab, int nsplit, long rowlen,
                                        int CW, int nb_main) {
  const int sg = threadIdx.x >> 6, l = threadIdx.x & 63;
  __shared__ float red[4][64];
  float g = 0.f;
  float* base = nullptr;
  long stride = 0, e = -1;
  if ((int)blockIdx.x < nb_main) {
    e = (long)blockIdx.x * 64 + l;                   // element of the [phase][rowlen] sums
    if (e < 4 * rowlen) {
      const long ph = e / rowlen, k = e - ph * rowlen;
      base = slab + ph * nsplit * rowlen + k;
      stride = rowlen;
    }
  } else {
    e = (long)((int)blockIdx.x - nb_main) * 64 + l;
    if (e < 4L * CW) {
      const long ph = e / CW, co = e - ph * CW;
      base = bslab + ph * nsplit * CW + co;
      stride = CW;
    }
  }
  if (base)
    for (int sp = sg; sp < nsplit; sp += 4) g += base[sp * stride];
  red[sg][l] = g;
  __syncthreads();
  if (sg == 0 && base) base[0] = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
}

// pass 2: dW[co][ci][r][s] = sum over the 4 phases of the phase tap (rr, ss) that (r, s) maps to
// (the map of wgrad_reduce_subpix_kernel), db = the 4 phase sums
__global__ void subpix_fold_kernel(const float* __restrict__ slab, const float* __restrict__ bslab, float* dw, float* db,
                                   int nsplit, int CW, int KW, int cout, int cin_valid, int lgCin, int nb_main) {
  const long rowlen = (long)CW * KW;
  if ((int)blockIdx.x < nb_main) {
    const long e = (long)blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= (long)cout * cin_valid * 9) return;
    const int rs = (int)(e % 9), ci = (int)((e / 9) % cin_valid), co = (int)(e / (9L * cin_valid));
    const int r = rs / 3, sc = rs % 3;
    float g = 0.f;
#pragma unroll
    for (int ph = 0; ph < 4; ++ph) {
      const int pa = ph >> 1, pb = ph & 1;
      const int rr = pa ? (r == 2) : (r > 0), ss = pb ? (sc == 2) : (sc > 0);
      g += slab[(long)ph * nsplit * rowlen + (long)co * KW + (((rr * 2 + ss) << lgCin) + ci)];
    }
    dw[e] = g;
  } else {
    const int co = ((int)blockIdx.x - nb_main) * blockDim.x + threadIdx.x;
    if (co >= cout) return;
    db[co] = (bslab[co] + bslab[(long)nsplit * CW + co]) + (bslab[2L * nsplit * CW + co] + bslab[3L * nsplit * CW + co]);
  }
}

// sum of the per-split slabs -> dW in the reference layout [co][ci][r][s] (+ db).  Block =
// 64 consecutive outputs x 4 split lanes (4 independent partial sums each), so that large
// split counts do not serialise on load latency; blocks >= nb_main reduce the bias slab.
// KSL: taps per row in the slab's k layout (KS, or 8 for the packed 7x7 rows of conv_halo_wgrad
// PK, whose s = 7 column is padding)
__global__ void wgrad_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ bslab,
                                    float* dw, float* db, int nsplit, int CW, int KW, int K,
                                    int cout, int cin_valid, int lgCin, int KS, int nb_main, int KSL) {
  const int sg = threadIdx.x >> 6, l = threadIdx.x & 63;
  __shared__ float red[4][64];
  float g = 0.f;
  bool valid;
  long dst = 0;
  const float* p = nullptr;
  long stride;
  if ((int)blockIdx.x < nb_main) {
    const long e = (long)blockIdx.x * 64 + l;
    const int co = (int)(e / K), k = (int)(e - (e / K) * K);
    const int tap = k >> lgCin, c = k & ((1 << lgCin) - 1);
    const int r = tap / KSL, sx = tap - (tap / KSL) * KSL;
    valid = e < (long)cout * K && c < cin_valid && sx < KS;
    dst = (((long)co * cin_valid + c) * KS + r) * KS + sx;
    p = slab + (long)co * KW + k;
    stride = (long)CW * KW;
  } else {
    const int co = ((int)blockIdx.x - nb_main) * 64 + l;
    valid = db != nullptr && co < cout;
    dst = co;
    p = bslab + co;
    stride = CW;
  }
  if (valid) {
    float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
    int s = sg;
    for (; s + 12 < nsplit; s += 16) {
      a0 += p[(long)s * stride];
      a1 += p[(long)(s + 4) * stride];
      a2 += p[(long)(s + 8) * stride];
      a3 += p[(long)(s + 12) * stride];
    }
    for (; s < nsplit; s += 4) a0 += p[(long)s * stride];
    g = (a0 + a1) + (a2 + a3);
  }
  red[sg][l] = g;
  __syncthreads();
  if (sg == 0 && valid) {
    const float t = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    if ((int)blockIdx.x < nb_main) dw[dst] = t;
    else db[dst] = t;
  }
}

// ----------------------------------------------------------------------------------------
// host dispatch
// ----------------------------------------------------------------------------------------
struct FwdTile { int bn, bm; };

FwdTile fwd_tile(int rows_needed) {
  if (rows_needed > 64) return {128, 128};
  if (rows_needed > 32) return {64, 128};
  if (rows_needed > 16) return {32, 128};
  return {16, 128};
}

int pad_pow2_8(int c) {
  int p = 8;
  while (p < c) p <<= 1;
  return p;
}

template <typename T, int KS, int WN, int WM, int RN, int RM>
int launch_fwd_t(const ConvArgs& a, int pro, int ups, int nblk, hipStream_t s) {
  dim3 g(nblk), b(64 * WN * WM);
  if (pro && ups) {
    if constexpr (KS == 3) hipLaunchKernelGGL((conv_fwd_kernel<T, KS, WN, WM, RN, RM, true, true>), g, b, 0, s, a);
    else return FV_E_UNSUPPORTED;
  } else if (pro) {
    if constexpr (KS != 7) hipLaunchKernelGGL((conv_fwd_kernel<T, KS, WN, WM, RN, RM, true, false>), g, b, 0, s, a);
    else return FV_E_UNSUPPORTED;
  } else if (ups) {
    if constexpr (KS == 3) hipLaunchKernelGGL((conv_fwd_kernel<T, KS, WN, WM, RN, RM, false, true>), g, b, 0, s, a);
    else return FV_E_UNSUPPORTED;
  } else {
    hipLaunchKernelGGL((conv_fwd_kernel<T, KS, WN, WM, RN, RM, false, false>), g, b, 0, s, a);
  }
  return FV_OK;
}

template <typename T, int KS>
int launch_fwd_ks(const ConvArgs& a, FwdTile t, int pro, int ups, int nblk, hipStream_t s) {
  if (t.bn == 128) return launch_fwd_t<T, KS, 2, 2, 4, 4>(a, pro, ups, nblk, s);
  if (t.bn == 64) return launch_fwd_t<T, KS, 2, 2, 2, 4>(a, pro, ups, nblk, s);
  if (t.bn == 32) return launch_fwd_t<T, KS, 2, 2, 1, 4>(a, pro, ups, nblk, s);
  return launch_fwd_t<T, KS, 1, 4, 1, 2>(a, pro, ups, nblk, s);
}

template <typename T>
int launch_fwd(const ConvArgs& a, int ks, FwdTile t, int pro, int ups, int nblk, hipStream_t s) {
  switch (ks) {
    case 1: return launch_fwd_ks<T, 1>(a, t, pro, ups, nblk, s);
    case 3: return launch_fwd_ks<T, 3>(a, t, pro, ups, nblk, s);
    case 7: return launch_fwd_ks<T, 7>(a, t, pro, ups, nblk, s);
  }
  return FV_E_UNSUPPORTED;
}

// v2 (DMA-fed bf16) path: bf16, no BN prologue, cin a multiple of 64, input < 2 GB
bool use_v2(const fv_conv_desc* d) {
  if (d->dtype != FV_BF16 || d->pro_act || d->cin % 64) return false;
  if (d->out_nchw_f32 || d->epi_sigmoid || d->cout % 8 || d->ldy % 8) return false;   // staged NHWC epilogue
  if (d->w % 8) return false;   // a DMA piece (8 pixels) must lie in one image row
  const long hin = d->upsample ? d->h / 2 : d->h, win = d->upsample ? d->w / 2 : d->w;
  return (long)d->n * hin * win * d->cin * 2 < (1L << 31);
}

// 3x3 halo path (conv3_halo_fwd2 / fwd3): co per block (256 / 128 / 64), 0 when not eligible
int halo3_bn(const fv_conv_desc* d) {
  if (!use_v2(d) || d->ksize != 3 || d->upsample || d->w % 64 || d->h % 4) return 0;
  if ((long)d->n * d->h * d->w * d->ldy * 2 >= (1L << 31)) return 0;
  // co % 256: the pipelined pair-of-taps kernel (3 % over conv_fwd_v2's 256 x 256 tile on
  // the res convs) -- unless its 256-pixel x 256-co tiles leave CUs idle (fewer tiles than the
  // 256 CUs, e.g. the 64x64 latent convs at B <= 8: the SURVEY 8(f) path's Generator), where the
  // 128-co tiles double the grid.  Only for >= 256 input channels (the latent-resolution
  // convs), so AFE.down2 (128 -> 256) keeps one kernel at every batch size.
  if (d->cout % 256 == 0)
    return d->cin < 256 || (long)d->n * (d->h / 4) * (d->w / 64) * (d->cout / 256) >= 256 ? 256 : 128;
  // AFE.down1's forward (64 -> 128 channels, K = 576): conv_fwd_v2's 128 x 256 tile measured
  // 500 us against 543 (pipelined halo) / 579 (single-tap halo) at 256x256, B=32
  // (r3, stage-major weights: still 527 vs 503 us in alternating convbench runs)
  if (d->cin == 64 && d->cout == 128) return 0;
  return d->cout % 128 == 0 ? 128 : d->cout % 64 == 0 ? 64 : 0;
}


// v2 tile configs: id -> (co per block, pixels per block); waves/layout in launch_v2_ks
struct V2Cfg { int bn, bm; };
constexpr V2Cfg kV2Cfg[] = {
    {128, 128},   // 0: 4 waves 2x2, wave 64co x 64px
    {64, 256},    // 1: 4 waves 1x4, wave 64co x 64px
    {16, 256},    // 2: 4 waves 1x4, wave 16co x 64px
    {256, 256},   // 3: 8 waves 4x2, wave 64co x 128px
    {128, 256},   // 4: 8 waves 2x4, wave 64co x 64px
    {256, 128},   // 5: 8 waves 4x2, wave 64co x 64px
};
int v2_cfg(int rows_needed) {
  if (rows_needed % 256 == 0) return 3;
  if (rows_needed > 64) return 0;
  if (rows_needed > 16) return 1;
  return 2;
}
FwdTile fwd_tile_v2(int rows_needed) {
  const V2Cfg c = kV2Cfg[v2_cfg(rows_needed)];
  return {c.bn, c.bm};
}
// rows of a prepared weight image (forward wk: cout; data-gradient wt: cin): a whole number
// of co tiles of EVERY kernel that may read it -- the v1 tiles (fwd_tile) and the v2 tiles
// (fwd_tile_v2) differ for 17..32 rows (32 vs 64), and the v2 kernels' weight DMA reads the
// whole tile (found by a 1x1 32 -> 128 conv's data gradient reading 32 rows past its wt).
int wrows(int rows_needed) {
  const int b1 = fwd_tile(rows_needed).bn, b2 = fwd_tile_v2(rows_needed).bn;
  const int b = b1 > b2 ? b1 : b2;
  return fv_cdiv(rows_needed, b) * b;
}

// mode: 0 plain, 1 upsample folded (KS 3), 2 sub-pixel phases (KS 2)
template <int KS, int WN, int WM, int RN, int RM, int BKS>
int launch_v2_b(const ConvArgs& a, int mode, int nblk, unsigned xb, hipStream_t s) {
  dim3 g(nblk), b(64 * WN * WM);
  if (mode == 3) {
    if constexpr (KS == 4) hipLaunchKernelGGL((conv_fwd_v2<KS, WN, WM, RN, RM, 3, BKS>), g, b, 0, s, a, xb);
    else return FV_E_UNSUPPORTED;
  } else if (mode == 2) {
    if constexpr (KS == 2) hipLaunchKernelGGL((conv_fwd_v2<KS, WN, WM, RN, RM, 2, BKS>), g, b, 0, s, a, xb);
    else return FV_E_UNSUPPORTED;
  } else if (mode == 1) {
    if constexpr (KS == 3) hipLaunchKernelGGL((conv_fwd_v2<KS, WN, WM, RN, RM, 1, BKS>), g, b, 0, s, a, xb);
    else return FV_E_UNSUPPORTED;
  } else {
    if constexpr (KS != 2 && KS != 4) hipLaunchKernelGGL((conv_fwd_v2<KS, WN, WM, RN, RM, 0, BKS>), g, b, 0, s, a, xb);
    else return FV_E_UNSUPPORTED;
  }
  return FV_OK;
}

// 4-wave tiles stage 32-deep k slices when K is short (<= 640) or the input is upsampled:
// there the 4-blocks-per-CU occupancy beats the deeper k step (A/B on the FaceVAE shapes)
template <int KS, int WN, int WM, int RN, int RM>
int launch_v2_t(const ConvArgs& a, int mode, int nblk, unsigned xb, hipStream_t s) {
  if constexpr (WN * WM == 4) {
    if (a.W % 16 == 0 && (a.Kpad <= 640 || mode != 0))
      return launch_v2_b<KS, WN, WM, RN, RM, 32>(a, mode, nblk, xb, s);
  }
  return launch_v2_b<KS, WN, WM, RN, RM, 64>(a, mode, nblk, xb, s);
}

template <int KS>
int launch_v2_ks(const ConvArgs& a, FwdTile t, int mode, int nblk, unsigned xb, hipStream_t s) {
  const int ups = mode;
  if (t.bn == 128 && t.bm == 128) return launch_v2_t<KS, 2, 2, 4, 4>(a, ups, nblk, xb, s);
  if (t.bn == 64) return launch_v2_t<KS, 1, 4, 4, 4>(a, ups, nblk, xb, s);
  if (t.bn == 16) return launch_v2_t<KS, 1, 4, 1, 4>(a, ups, nblk, xb, s);
  if (t.bn == 256 && t.bm == 256) return launch_v2_t<KS, 4, 2, 4, 8>(a, ups, nblk, xb, s);
  if (t.bn == 128 && t.bm == 256) return launch_v2_t<KS, 2, 4, 4, 4>(a, ups, nblk, xb, s);
  if (t.bn == 256 && t.bm == 128) return launch_v2_t<KS, 4, 2, 4, 4>(a, ups, nblk, xb, s);
  return FV_E_UNSUPPORTED;
}

int launch_v2(const ConvArgs& a, int ks, FwdTile t, int ups, int nblk, unsigned xb, hipStream_t s) {
  switch (ks) {
    case 2: return launch_v2_ks<2>(a, t, 2, nblk, xb, s);       // sub-pixel phases only
    case 4: return launch_v2_ks<4>(a, t, 3, nblk, xb, s);       // stride-2 low-res dgrad only
    case 1: return launch_v2_ks<1>(a, t, ups, nblk, xb, s);
    case 3: return launch_v2_ks<3>(a, t, ups, nblk, xb, s);
    case 7: return launch_v2_ks<7>(a, t, ups, nblk, xb, s);
  }
  return FV_E_UNSUPPORTED;
}

// upsample + 3x3 conv as 4 sub-pixel phases of a 2x2 conv over the low-res input (bf16 v2
// path; FV_DISABLE_SUBPIX=1 keeps the folded-upsample 3x3 kernel).  2.25x fewer MACs than the
// reference formulation (reported utilisation still uses the reference FLOPs).
static int g_disable_subpix = -1;
bool use_subpix(const fv_conv_desc* d) {
  if (g_disable_subpix < 0) {
    const char* e = getenv("FV_DISABLE_SUBPIX");
    g_disable_subpix = (e && e[0] == '1') ? 1 : 0;
  }
  if (g_disable_subpix || !d->upsample || d->ksize != 3 || !use_v2(d)) return false;
  const int hl = d->h / 2, wl = d->w / 2;
  if (fv_ilog2(hl) < 0 || fv_ilog2(wl) < 0 || wl % 16) return false;
  const long pl = (long)d->n * hl * wl;
  return pl % fwd_tile_v2(d->cout).bm == 0;
}

// the 64-channel co tile on conv3_halo_fwd3 (8 waves, 8-row tiles); FV_C64T=0 keeps
// conv3_halo_fwd2<1, 4, 4, 4, 3> (A/B).  Read per call.
static bool c64t_on() {
  const char* e = getenv("FV_C64T");
  return !(e && e[0] == '0');
}

// SIMD-partner schedule of the halo 3x3 kernels (conv3_halo_fwd3 / conv3_halo_fp8 SCH):
// FV_RES_SCHED = 0 (prio flips, lockstep), 1 (static prio for waves 4-7), 2 (stagger), 3
// (both); unset: the measured default of each kernel (dflt).  conv3_halo_fwd3 keeps 0 and 2
// (1 / 3 measured no better, below).  Read per call (tests compare the
// schedules bit for bit in one process).  r5, alternating convbench runs on one box, B=32 bf16
// res fwd / dgrad: 0: 130 / 122, 1: 124 / 118, 2: 120 / 115, 3: 126 / 119 us; B=64 fp8 res
// fwd / dgrad: 0: 175 / 166, 1: 173 / 163, 2: 172 / 155, 3: 165 / 155 us.
// data-parallel fp8 (fv_fp8_set_deferred_roll): the *_site convs leave the in-flight amax in the
// site; the caller all-reduces (MAX) every site's amax once per step and rolls them together
static int g_fp8_defer_roll = 0;

static int res_sched(int dflt) {
  const char* e = getenv("FV_RES_SCHED");
  return (e && e[0] >= '0' && e[0] <= '3') ? e[0] - '0' : dflt;
}

// data gradient of an upsample + 3x3 conv computed directly at the low resolution as a
// stride-2 4x4 conv over dy (bf16 v2 path; replaces dgrad at the high resolution followed by
// the 2x2 sum of fv_upsample2x_bwd: 0.44x the MACs, one pass fewer)
bool use_dgrad_lowres(const fv_conv_desc* d) {
  if (g_disable_subpix < 0) use_subpix(d);     // reads FV_DISABLE_SUBPIX
  if (g_disable_subpix || !d->upsample || d->ksize != 3 || d->dtype != FV_BF16) return false;
  const int ct = pad_pow2_8(d->cout);
  if (ct % 64 || d->cin % 8 || (d->w / 2) % 16) return false;
  return (long)d->n * d->h * d->w * ct * 2 < (1L << 31);
}

// UpBlock2D convs on the halo kernel (conv3_halo_fwd3 MODE 1 forward, MODE 2 low-res data
// gradient); FV_UP_HALO=0 keeps conv_fwd_v2 MODE 2 / 3 (A/B).  Read per call.
static bool up_halo_on() {
  const char* e = getenv("FV_UP_HALO");
  return !(e && e[0] == '0');
}
// UpBlock2D forward with a 128-channel input on the sliding-band kernel (conv3up_band_fwd;
// FV_UPBAND=0: the halo kernel's MODE 1, A/B).  Its weights are the plain sub-pixel layout.
static bool use_upband(const fv_conv_desc* d) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("FV_UPBAND");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  if (!on || d->dtype != FV_BF16 || !use_subpix(d)) return false;
  const int hl = d->h / 2, wl = d->w / 2;
  return d->cin == 128 && d->cin_valid == 128 && d->cout % 64 == 0 && wl % 32 == 0 && hl % 8 == 0 &&
         !d->out_nchw_f32 && !d->epi_sigmoid && !d->pro_act && d->ldy % 8 == 0 &&
         (long)d->n * hl * wl * 128 * 2 < (1L << 31) && (long)d->n * d->h * d->w * d->ldy * 2 < (1L << 31);
}
static bool use_subpix_halo(const fv_conv_desc* d) {
  if (!up_halo_on() || !use_subpix(d) || use_upband(d)) return false;
  const int hl = d->h / 2, wl = d->w / 2;
  return d->cout % 64 == 0 && d->cin % 32 == 0 && d->cin >= 64 && d->cin_valid == d->cin && wl % 64 == 0 &&
         hl % 4 == 0 && !d->out_nchw_f32 && !d->epi_sigmoid && !d->pro_act && d->ldy % 8 == 0 &&
         (long)d->n * hl * wl * d->cin * 2 < (1L << 31) && (long)d->n * d->h * d->w * d->ldy * 2 < (1L << 31);
}
// co tile (256 / 128 rows) of the low-res data gradient on the halo kernel, 0 = not on it
static int dgrad_halo_bn(const fv_conv_desc* d) {
  if (!up_halo_on() || !use_dgrad_lowres(d)) return 0;
  const int hl = d->h / 2, wl = d->w / 2;
  if (pad_pow2_8(d->cout) != d->cout || d->cout % 32 || wl % 64 || hl % 4 || d->cin_valid != d->cin) return 0;
  if ((long)d->n * d->h * d->w * d->cout * 2 >= (1L << 31)) return 0;
  return d->cin % 256 == 0 ? 256 : d->cin % 128 == 0 ? 128 : 0;
}
// elements of the phase weight images (weight_prep_phase_kernel): the one size both the
// queries and the launches use
static long phase_wk_elems(const fv_conv_desc* d) { return 4L * (d->cin / 32) * 4 * d->cout * 32; }
static long phase_wt_elems(const fv_conv_desc* d) { return 4L * (4 * d->cout / 32) * d->cin * 32; }

// Generator.out_conv shape: 7x7, 64 -> <= 4 channels, NCHW fp32 output (bf16 operands)
bool use_c7n(const fv_conv_desc* d) {
  return d->dtype == FV_BF16 && d->ksize == 7 && d->cin == 64 && d->cin_valid == 64 &&
         d->cout <= 4 && !d->pro_act && !d->upsample && d->w % 64 == 0 && d->h % C7_TR == 0 &&
         (long)d->n * d->h * d->w * 64 * 2 < (1L << 31);
}

// band of output rows per block of the sliding out_conv forward (conv7_n3_fwd2): the largest
// of 128/64/32/16/8/4 dividing H that still gives >= 256 blocks (else the smallest dividing;
// use_c7n guarantees H % 4 == 0).  FV_C7_BAND=b forces a band (tests: multi-group rings on
// small images); read per call.
static int c7n_band(const fv_conv_desc* d) {
  if (const char* e = getenv("FV_C7_BAND")) {
    const int b = atoi(e);
    if (b >= 4 && b % 4 == 0 && d->h % b == 0) return b;
  }
  int pick = 0;
  for (int band : {128, 64, 32, 16, 8, 4}) {
    if (d->h % band) continue;
    pick = band;
    if ((long)d->n * (d->w / 64) * (d->h / band) >= 256) return band;
  }
  return pick;
}

// 3x3 weight gradient with the halo-staged input, rows sliding down a segment
// (conv3_halo_wgrad2; its tile-per-row-segment predecessor ran 518 us against 262 us for
// AFE.down1)
static int g_h3w_all = -1;
bool use_h3w(const fv_conv_desc* d) {
  // measured against conv_wgrad_v2 (tools/convbench.py): 12 % faster on AFE.down1 (64 -> 128,
  // whose v2 tile is 128 x 128).  Wider inputs run it as 64-channel input tiles (r4: the res /
  // down2 weight gradients; FV_H3W_ALL=0 keeps them on conv_wgrad_v2 for A/B)
  if (g_h3w_all < 0) {
    const char* e = getenv("FV_H3W_ALL");
    g_h3w_all = (e && e[0] == '0') ? 0 : 1;
  }
  const bool cin_ok = d->cin == 64 || (g_h3w_all && d->cin % 64 == 0);
  // (a BN-apply prologue runs the generic kernels: its fast variants, "option B", were removed in r6)
  if (d->pro_act) return false;
  return d->dtype == FV_BF16 && d->ksize == 3 && !d->upsample && cin_ok &&
         d->cin_valid == d->cin && d->cout % 128 == 0 && d->w % 64 == 0;
}

// out_conv weight gradient as "row taps in N" (conv7_n3_wgrad)
bool use_c7w(const fv_conv_desc* d) {
  return d->dtype == FV_BF16 && d->ksize == 7 && d->cin == 64 && d->cin_valid == 64 &&
         d->cout <= 4 && !d->pro_act && !d->upsample && d->w % 64 == 0 &&
         (long)d->n * d->h * d->w * 64 * 2 < (1L << 31);
}

int check_desc(const fv_conv_desc* d) {
  FV_REQUIRE(d, "null conv descriptor");
  FV_REQUIRE(d->dtype == FV_F32 || d->dtype == FV_BF16, "conv dtype must be f32 or bf16");
  FV_REQUIRE(d->ksize == 1 || d->ksize == 3 || d->ksize == 7, "ksize must be 1, 3 or 7");
  FV_REQUIRE(d->n > 0 && d->h > 0 && d->w > 0, "bad spatial size");
  FV_REQUIRE(fv_ilog2(d->cin) >= 3, "cin must be a power of two >= 8 (got %d)", d->cin);
  FV_REQUIRE(d->cin_valid > 0 && d->cin_valid <= d->cin, "bad cin_valid");
  FV_REQUIRE(d->cout > 0, "bad cout");
  FV_REQUIRE(!d->upsample || (d->h % 2 == 0 && d->w % 2 == 0), "upsample needs even h, w");
  FV_REQUIRE(!d->upsample || d->ksize == 3, "upsample only with 3x3");
  FV_REQUIRE(!d->pro_act || d->ksize != 7, "BN prologue not supported for 7x7");
  FV_REQUIRE(!d->pro_act || fv_slope_ok(d->pro_slope), "prologue slope must be in [0, 1] (got %g)", (double)d->pro_slope);
  return FV_OK;
}

int kpad_of(int ks, int cin) { return fv_cdiv((long)ks * ks * cin, BK) * BK; }

// 7x7 halo wgrad: in_conv (cin 8 -> 64, dy stride 64) or out_conv (cin 64 -> cout <= 8, dy stride 8)
// the in_conv weight gradient in the packed k layout (conv_halo_wgrad PK); FV_WG7_PACK=0 keeps
// the 8-channel padded layout (A/B).  Read per call.
static bool halo_wg_pk(const fv_conv_desc* d) {
  const char* e = getenv("FV_WG7_PACK");
  if (e && e[0] == '0') return false;
  return d->ksize == 7 && d->cin == 8 && d->cin_valid <= 4;
}
static int halo_wg_tr(const fv_conv_desc* d) {
  if (d->ksize != 7 || d->upsample || d->pro_act || d->w % 64) return 0;
  int tr = 0;
  if (d->cin == 8 && d->cout == 64) tr = 4;
  else if (d->cin == 64 && d->cout <= 8) tr = 2;
  return (tr && d->h % tr == 0) ? tr : 0;
}

// wgrad plan: v2 (bf16 DMA-fed, 8 waves), halo (7x7), or the register-staged v1 (fp32 / BN prologue)
struct WgPlan {
  int v2, bkt, bc, px, ntk, ntc, nsplit, nsteps, sps, KW, CW, cfg, sub;
};

// wgrad v2 tile configs: k rows x co cols per block, 8 waves as wk x wc, pixels per stage,
// LDS ring depth.  The 32-B-block XOR swizzle of the transposed images needs bkt % 128 == 0.
struct Wg2Cfg { int bkt, bc, wk, wc, px, ns; };
constexpr Wg2Cfg kWg2Cfg[] = {
    {256, 256, 2, 4, 64, 2},   // 0  (64 KB stages)
    {128, 256, 2, 4, 64, 3},   // 1
    {256, 128, 4, 2, 64, 3},   // 2
    {128, 128, 2, 4, 64, 4},   // 3
    {128, 64, 8, 1, 64, 4},    // 4
    {256, 16, 8, 1, 64, 2},    // 5
    {256, 256, 2, 4, 32, 4},   // 6  (32 KB stages, 3 in flight)
    {384, 64, 8, 1, 64, 2},    // 7
    {384, 64, 4, 2, 64, 2},    // 8
    {128, 128, 2, 4, 32, 4},   // 9
    {256, 128, 4, 2, 32, 4},   // 10
    {256, 64, 8, 1, 64, 3},    // 11 (sub-pixel phases of the 64-channel up conv, K = 512)
    {512, 64, 8, 1, 64, 2},    // 12
};
constexpr int kNumWg2Cfg = sizeof(kWg2Cfg) / sizeof(kWg2Cfg[0]);
int wg2_cfg(const fv_conv_desc* d, int K) {
  const int bc = d->cout > 128 ? 256 : d->cout > 64 ? 128 : d->cout > 16 ? 64 : 16;
  // FV_WG1_CFG=c: tile config c (0..5) for the 1x1 weight gradients (A/B; read per call)
  if (d->ksize == 1) {
    const char* e = getenv("FV_WG1_CFG");
    if (e && e[0] >= '0' && e[0] <= '5') {
      const int c = e[0] - '0';
      if (d->cout % kWg2Cfg[c].bc == 0 && K % kWg2Cfg[c].bkt == 0) return c;
    }
  }
  // defaults from the FaceVAE-shape tile sweep (r1): 384 x 64 tiles for the
  // 64-channel layers (K = 1152 splits exactly), 32-pixel stages 3-deep when K is not a
  // multiple of 256 at 256 channels
  if (bc == 16) return 5;
  if (bc == 64) return (K % 384 == 0 && d->w % 64 == 0) ? 7 : 4;
  const bool k256 = fv_cdiv(K, 256) * 256 <= fv_cdiv(K, 128) * 128;
  // (r3, alternating convbench runs on one box, res wgrad at B=32: cfg 0 150-153 us, cfg 6
  // (32-pixel stages, 3 in flight) 168, cfg 1 (128 x 256 tiles, 3 stages) 202-207)
  if (bc == 256) return K % 256 == 0 ? 0 : (d->ksize == 3 && d->w % 32 == 0 ? 6 : 1);
  return k256 ? 2 : 3;
}
// UpBlock2D weight gradient on conv3_up_wgrad: bf16 nearest-x2 + 3x3, 64-channel multiples,
// 64-column output strips (FV_UPW=0: the conv_wgrad_v2 sub-pixel path, A/B)
static bool use_upw(const fv_conv_desc* d) {
  static int on = -1;
  if (on < 0) {
    const char* e = getenv("FV_UPW");
    on = (e && e[0] == '0') ? 0 : 1;
  }
  return on && d->dtype == FV_BF16 && d->upsample && d->ksize == 3 && !d->pro_act && d->cin % 64 == 0 &&
         d->cin_valid == d->cin && d->cout % 64 == 0 && d->w % 64 == 0 && d->h % 4 == 0;
}
// an integer tuning knob from the environment (A/B runs), read per call
static int env_int(const char* name, int dflt) {
  const char* e = getenv(name);
  const int v = e ? atoi(e) : 0;
  return v > 0 ? v : dflt;
}

WgPlan plan_wgrad(const fv_conv_desc* d) {
  WgPlan p{};
  const int K = d->ksize * d->ksize * d->cin;
  const long P = (long)d->n * d->h * d->w;
  const long hin = d->upsample ? d->h / 2 : d->h, win = d->upsample ? d->w / 2 : d->w;
  // 32-bit buffer offsets: x and dy (channel stride = cout padded to a power of two >= 8, as
  // every caller passes; fv_conv2d_bwd_weight re-checks the real stride) must stay < 2 GB
  const bool fits = d->dtype == FV_BF16 && (long)d->n * hin * win * d->cin * 2 < (1L << 31) &&
                   P * pad_pow2_8(d->cout) * 2 < (1L << 31);
  p.v2 = fits && !d->pro_act;
  // out_conv 7x7 64 -> <= 4 (v2 == 3): blocks = (image, 64-column strip, row segment), about
  // 2 per CU (r6: 1024 -> 512 blocks halves the 58.7 MB of slabs; out_conv weight gradient
  // 98.4 -> 90.4 us + reduce 15 -> 10.6 us, step -0.03 ms; 256 blocks: 114 us;
  // profiles/r6/r6k_ab_wgrad_blocks.log); slab [block][32 (r, co)][448 (s, ci)]
  if (p.v2 && use_c7w(d)) {
    const int strips = d->w / 64;
    int nseg = fv_cdiv(env_int("FV_C7W_BLOCKS", 512), d->n * strips);
    if (nseg > fv_cdiv(d->h, 8)) nseg = fv_cdiv(d->h, 8);
    if (nseg < 1) nseg = 1;
    p.v2 = 3;
    p.sps = fv_cdiv(d->h, nseg);                 // rows per segment
    p.nsteps = fv_cdiv(d->h, p.sps);             // segments
    p.nsplit = d->n * strips * p.nsteps;
    p.CW = 32;
    p.KW = 448;
    p.ntk = p.ntc = 1;
    return p;
  }
  // 3x3 sliding-row wgrad (v2 == 5, conv3_halo_wgrad2): blocks = (image, 64-column strip,
  // row segment) x co tiles of 128, ~1 block per CU; splits = image x strip x segment
  if (fits && use_h3w(d)) {
    const int strips = d->w / 64;
    p.v2 = 5;
    p.ntc = d->cout / 128;
    p.ntk = d->cin / 64;               // 64-channel input tiles
    int nseg = (256 / (p.ntc * p.ntk) + d->n * strips / 2) / (d->n * strips);
    if (nseg < 1) nseg = 1;
    if (nseg > d->h / 4) nseg = d->h / 4 > 0 ? d->h / 4 : 1;
    p.sps = fv_cdiv(d->h, nseg);                  // rows per segment
    p.nsteps = fv_cdiv(d->h, p.sps);              // segments
    p.nsplit = d->n * strips * p.nsteps;
    p.CW = d->cout;
    p.KW = K;
    return p;
  }
  // 7x7 halo path (v2 == 2): one persistent block per CU, ntk = 1 (all k in one tile)
  const int htr = halo_wg_tr(d);
  if (p.v2 && htr) {
    const int nt = d->cin == 8 ? 4 : 1;
    p.v2 = 2;
    p.bkt = halo_wg_pk(d) ? 7 * 32 : fv_cdiv(K, 16) * 16;
    p.bc = nt * 16;
    p.px = htr * 64;
    p.ntk = 1;
    p.ntc = 1;
    p.nsteps = (int)(P / p.px);                  // pixel tiles
    p.nsplit = p.nsteps < 256 ? p.nsteps : 256;  // persistent blocks
    p.sps = fv_cdiv(p.nsteps, p.nsplit);
    p.KW = p.bkt;
    p.CW = p.bc;
    return p;
  }
  if (fits && use_upw(d)) {
    // sub-pixel sliding-row weight gradient (v2 == 6, conv3_up_wgrad): blocks = (co tile, ci
    // tile) x splits of `sps` consecutive (image, 64-column output strip) units, ~one block per
    // CU; slab [phase][split][co][4 cin] as the v2 sub-pixel path
    p.sub = 1;
    p.v2 = 6;
    p.ntc = d->cout / 64;
    p.ntk = d->cin / 64;
    const int units = d->n * (d->w / 64), tiles = p.ntc * p.ntk;
    p.sps = (units * tiles + 128) / 256;
    // FV_UPW_SPB=k: k units per block (tests: ragged last split at small shapes)
    if (const char* e = getenv("FV_UPW_SPB")) p.sps = atoi(e);
    if (p.sps < 1) p.sps = 1;
    p.nsteps = units;
    p.nsplit = fv_cdiv(units, p.sps);
    p.CW = d->cout;
    p.KW = 4 * d->cin;
    return p;
  }
  if (p.v2 && use_subpix(d) && (d->w / 2) % 64 == 0) {
    // weight gradient of the 4 sub-pixel phases (2x2 taps over the low-res input, 0.44x the
    // MACs of the upsampled 3x3 formulation); wgrad_reduce folds the phases back into 3x3
    p.sub = 1;
    p.cfg = d->cout > 64 ? (d->cout > 128 ? 0 : 2) : 11;
    const Wg2Cfg& c = kWg2Cfg[p.cfg];
    p.bkt = c.bkt;
    p.bc = c.bc;
    p.px = c.px;
    const int K2 = 4 * d->cin;
    const long P2 = (long)d->n * (d->h / 2) * (d->w / 2);
    p.ntk = fv_cdiv(K2, p.bkt);
    p.ntc = fv_cdiv(d->cout, p.bc);
    p.nsteps = (int)(P2 / p.px);
    const int ntile = p.ntk * p.ntc;
    int ns = (64 + ntile / 2) / ntile;         // x4 phases ~ one block per CU
    if (ns < 1) ns = 1;
    if (ns > p.nsteps) ns = p.nsteps;
    p.sps = fv_cdiv(p.nsteps, ns);
    p.nsplit = fv_cdiv(p.nsteps, p.sps);
    p.KW = p.ntk * p.bkt;
    p.CW = p.ntc * p.bc;
    return p;
  }
  if (p.v2) {
    p.cfg = wg2_cfg(d, K);
    const Wg2Cfg& c = kWg2Cfg[p.cfg];
    p.bkt = c.bkt;
    p.bc = c.bc;
    p.px = c.px;
  } else {
    p.bc = d->cout > 64 ? 128 : (d->cout > 16 ? 64 : 16);
    p.bkt = 128;
    p.px = 32;
  }
  p.ntk = fv_cdiv(K, p.bkt);
  p.ntc = fv_cdiv(d->cout, p.bc);
  p.nsteps = fv_cdiv(P, p.px);
  const int ntile = p.ntk * p.ntc;
  const int wblk = env_int("FV_WG2_BLOCKS", 256);   // (128: 1x1 weight gradients 45 / 33 -> 67 / 40 us)
  int ns = p.v2 ? (wblk + ntile / 2) / ntile : 768 / ntile;
  if (ns < 1) ns = 1;
  if (ns > p.nsteps) ns = p.nsteps;
  p.sps = fv_cdiv(p.nsteps, ns);
  p.nsplit = fv_cdiv(p.nsteps, p.sps);
  p.KW = p.ntk * p.bkt;
  p.CW = p.ntc * p.bc;
  return p;
}

template <int KS, int CFG>
int launch_wg2_t(const Wg2Args& a, int ups, int nblk, hipStream_t s) {
  constexpr Wg2Cfg c = kWg2Cfg[CFG];
  if constexpr (KS == 2) {     // sub-pixel phases only
    if constexpr (CFG == 0 || CFG == 2 || CFG == 11 || CFG == 12) {
      hipLaunchKernelGGL((conv_wgrad_v2<2, c.bkt, c.bc, c.wk, c.wc, c.px, c.ns, false, true>), dim3(nblk), dim3(512), 0,
                         s, a);
      return FV_OK;
    } else {
      return FV_E_UNSUPPORTED;
    }
  } else {
  if (ups) {
    if constexpr (KS == 3)
      hipLaunchKernelGGL((conv_wgrad_v2<KS, c.bkt, c.bc, c.wk, c.wc, c.px, c.ns, true>), dim3(nblk), dim3(512), 0, s, a);
    else return FV_E_UNSUPPORTED;
  } else {
    hipLaunchKernelGGL((conv_wgrad_v2<KS, c.bkt, c.bc, c.wk, c.wc, c.px, c.ns, false>), dim3(nblk), dim3(512), 0, s, a);
  }
  return FV_OK;
  }
}

template <int KS, int CFG = 0>
int launch_wg2_ks(const Wg2Args& a, const WgPlan& p, int ups, int nblk, hipStream_t s) {
  if constexpr (CFG < kNumWg2Cfg) {
    if constexpr (KS != 3 && KS != 2 && CFG > 5) return FV_E_UNSUPPORTED;   // experiment configs: 3x3 only
    if (p.cfg == CFG) return launch_wg2_t<KS, CFG>(a, ups, nblk, s);
    return launch_wg2_ks<KS, CFG + 1>(a, p, ups, nblk, s);
  }
  return FV_E_UNSUPPORTED;
}

int launch_wg2(const Wg2Args& a, int ks, const WgPlan& p, int ups, int nblk, hipStream_t s) {
  if (p.sub) return launch_wg2_ks<2>(a, p, 0, nblk, s);
  switch (ks) {
    case 1: return launch_wg2_ks<1>(a, p, ups, nblk, s);
    case 3: return launch_wg2_ks<3>(a, p, ups, nblk, s);
    case 7: return launch_wg2_ks<7>(a, p, ups, nblk, s);
  }
  return FV_E_UNSUPPORTED;
}

template <typename T, int KS, int WK, int WC, int RK, int RC>
int launch_wg_t(const WgArgs& a, int pro, int ups, int nblk, hipStream_t s) {
  dim3 g(nblk), b(64 * WK * WC);
  if (pro && ups) {
    if constexpr (KS == 3) hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, WK, WC, RK, RC, true, true>), g, b, 0, s, a);
    else return FV_E_UNSUPPORTED;
  } else if (pro) {
    if constexpr (KS != 7) hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, WK, WC, RK, RC, true, false>), g, b, 0, s, a);
    else return FV_E_UNSUPPORTED;
  } else if (ups) {
    if constexpr (KS == 3) hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, WK, WC, RK, RC, false, true>), g, b, 0, s, a);
    else return FV_E_UNSUPPORTED;
  } else {
    hipLaunchKernelGGL((conv_wgrad_kernel<T, KS, WK, WC, RK, RC, false, false>), g, b, 0, s, a);
  }
  return FV_OK;
}

template <typename T, int KS>
int launch_wg_ks(const WgArgs& a, const WgPlan& t, int pro, int ups, int nblk, hipStream_t s) {
  if (t.bc == 128) return launch_wg_t<T, KS, 2, 2, 4, 4>(a, pro, ups, nblk, s);
  if (t.bc == 64) return launch_wg_t<T, KS, 2, 2, 4, 2>(a, pro, ups, nblk, s);
  return launch_wg_t<T, KS, 4, 1, 2, 1>(a, pro, ups, nblk, s);
}

template <typename T>
int launch_wg(const WgArgs& a, int ks, const WgPlan& t, int pro, int ups, int nblk, hipStream_t s) {
  switch (ks) {
    case 1: return launch_wg_ks<T, 1>(a, t, pro, ups, nblk, s);
    case 3: return launch_wg_ks<T, 3>(a, t, pro, ups, nblk, s);
    case 7: return launch_wg_ks<T, 7>(a, t, pro, ups, nblk, s);
  }
  return FV_E_UNSUPPORTED;
}

}  // namespace

extern "C" {

size_t fv_conv_wk_elems(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  const size_t rows = (size_t)wrows(d->cout);
  if (use_c7n(d)) return 32 * 448;
  if (use_subpix_halo(d)) return (size_t)phase_wk_elems(d);
  if (use_subpix(d)) return 4 * rows * kpad_of(2, d->cin);
  return rows * kpad_of(d->ksize, d->cin);
}

size_t fv_conv_wt_elems(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  const int cin_t = pad_pow2_8(d->cout);
  const size_t rows = (size_t)wrows(d->cin);
  if (dgrad_halo_bn(d)) return (size_t)phase_wt_elems(d);
  if (use_dgrad_lowres(d)) return rows * 16 * cin_t;
  return rows * kpad_of(d->ksize, cin_t);
}

int fv_conv2d_dgrad_lowres(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  return use_dgrad_lowres(d) ? 1 : 0;
}

// 7x7 halo path: (cin 8 -> cout 64, TR 8, weights in LDS) or (cin 64 -> cout <= 16, TR 2)
static int halo_tr(const fv_conv_desc* d) {
  if (d->dtype != FV_BF16 || d->ksize != 7 || d->pro_act || d->upsample || d->w % 64) return 0;
  int tr = 0;
  // (8-row tiles for the 8-channel side, 16 MFMAs per 8 LDS reads per wave, measured 13.28 ->
  // 13.33 ms/step in an A/B: not kept)
  if (d->cin == 8 && d->cout == 64) tr = 4;
  else if (d->cin == 64 && d->cout <= 16) tr = 2;
  if (!tr || d->h % tr) return 0;
  if ((long)d->n * d->h * d->w * d->cin * 2 >= (1L << 31)) return 0;
  return tr;
}

// the launch of forward-conv descriptor fd runs conv7c4_fwd (packed 7x7 weights, smaj 2)
static bool use_c74(const fv_conv_desc* fd) {
  return halo_tr(fd) == 4 && fd->cin == 8 && fd->cin_valid <= 4 && fd->cout == 64 && fd->ldy == 64 &&
         !fd->epi_sigmoid && !fd->out_nchw_f32;
}
// conv7c4_fwd's persistent grid: G blocks (<= 512, two per CU) of c74_tiles_per_block tiles
// each (block b: tiles b, b + G, ...); G = the BN record count (one record per block)
static int c74_tiles_per_block(const fv_conv_desc* d) {
  const int ntiles = d->n * (d->h / C74_TR) * (d->w / 64);
  return fv_cdiv(ntiles, 512);
}
static int c74_grid(const fv_conv_desc* d) {
  return fv_cdiv(d->n * (d->h / C74_TR) * (d->w / 64), c74_tiles_per_block(d));
}
// the launch of forward-conv descriptor fd runs conv3c64_fwd (64 input channels, sliding band,
// weights in registers; plain [co][Kpad] weights)
static bool use_c64(const fv_conv_desc* fd) {
  return fd->dtype == FV_BF16 && fd->ksize == 3 && !fd->upsample && !fd->pro_act && fd->cin == 64 &&
         fd->cin_valid == 64 && fd->cout % 64 == 0 && fd->ldy % 8 == 0 && !fd->epi_sigmoid && !fd->out_nchw_f32 &&
         fd->w % 64 == 0 && fd->h % 32 == 0 && (long)fd->n * fd->h * fd->w * 64 * 2 < (1L << 31) &&
         (long)fd->n * fd->h * fd->w * fd->ldy * 2 < (1L << 31);
}
// bands per (image, strip, 64-channel group): about one block per CU, bands of 32k rows
static int c64_bands(const fv_conv_desc* d) {
  const long base = (long)d->n * (d->w / 64) * (d->cout / 64);
  int nb = 1;
  while (base * nb < 256 && d->h % (nb * 64) == 0) nb *= 2;
  return nb;
}
static FwdTile plan_tile(const fv_conv_desc* d) {
  const int tr = halo_tr(d);
  if (tr) return {d->cout <= 16 ? 16 : 64, tr * 64};
  return use_v2(d) ? fwd_tile_v2(d->cout) : fwd_tile(d->cout);
}

// pixels per BN-statistics record = the pixels of one wave row of the tile (BM / WM)
static int stats_record_pixels(const fv_conv_desc* d) {
  if (use_c7n(d)) return 64;
  if (use_upband(d)) return UPB_G * 2 * 32;                  // (block, 4 iterations, phase)
  if (use_subpix_halo(d)) return 128;                         // (tile, wave row, phase): RM * 16                                  // one 64-pixel row segment
  if (use_c74(d)) return c74_tiles_per_block(d) * C74_TR * 64;   // one record per block
  if (use_c64(d)) return C64_G * 64;                          // 8 iterations x one wave's row
  if (halo_tr(d)) return plan_tile(d).bm / 8;                 // 8 waves stacked over pixels
  const FwdTile t = plan_tile(d);
  if (const int bn = halo3_bn(d)) return bn == 256 ? 128 : 64;   // RM * 16 pixels per wave row
  if (use_v2(d)) {
    if (t.bn == 64 || t.bn == 16 || (t.bn == 128 && t.bm == 256)) return t.bm / 4;
    return t.bm / 2;                                          // 128x128, 256x256, 256x128
  }
  return t.bn == 16 ? t.bm / 4 : t.bm / 2;                    // v1 layouts (launch_fwd_ks)
}

int fv_conv2d_stats_block_pixels(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  return stats_record_pixels(d);
}

int fv_conv2d_stats_blocks(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  return fv_cdiv((long)d->n * d->h * d->w, stats_record_pixels(d));
}

static fv_conv_desc dgrad_desc(const fv_conv_desc* d);

// the launch of forward-conv descriptor fd runs a halo 3x3 kernel (conv_run's halo3 branch:
// conv3_halo_fwd3 / fwd2), whose weights are prepared stage-major (weight_prep_body smaj) with
// wk_rows(fd) rows per tap unit
static bool h3s_layout(const fv_conv_desc* fd) {
  return !use_c7n(fd) && !halo_tr(fd) && !use_subpix(fd) && !use_c64(fd) && halo3_bn(fd) != 0;
}
static int wk_rows(const fv_conv_desc* fd) {
  return wrows(fd->cout);
}
static int lay_of(const fv_conv_desc* fd) { return use_c74(fd) ? 2 : h3s_layout(fd) ? 1 : 0; }
// ... for the forward weights (wk) and the data gradient's transposed weights (wt) of conv d
static int smaj_wk(const fv_conv_desc* d) { return lay_of(d); }
static int smaj_wt(const fv_conv_desc* d) {
  if (use_dgrad_lowres(d)) return 0;
  const fv_conv_desc t = dgrad_desc(d);
  return lay_of(&t);
}
// row length of a prepared image: the packed 7x7 layout's rows are C74_K long
static int kpad_lay(int lay, int kpad) { return lay == 2 ? C74_K : kpad; }

int fv_conv_weight_prep(const fv_conv_desc* d, const float* w_param, const float* sigma, void* wk,
                        void* wt, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  hipStream_t s = (hipStream_t)stream;
  const int ks = d->ksize;
  const bool generic_wk = wk && !use_c7n(d) && !use_subpix(d);
  const bool generic_wt = wt && !use_dgrad_lowres(d);
  if (generic_wk && generic_wt) {
    // the common case: forward and transposed layouts in one launch
    const int cin_t = pad_pow2_8(d->cout);
    WPrepJob j0{wk, wrows(d->cout), kpad_lay(smaj_wk(d), kpad_of(ks, d->cin)), fv_ilog2(d->cin),
                ks * ks * d->cin, 0, 0, smaj_wk(d)};
    WPrepJob j1{wt, wrows(d->cin), kpad_lay(smaj_wt(d), kpad_of(ks, cin_t)), fv_ilog2(cin_t),
                ks * ks * cin_t, 1, 0, smaj_wt(d)};
    j0.nb = (int)std::min<long>(fv_cdiv((long)j0.rows * j0.Kpad, 256), 4096);
    j1.nb = (int)std::min<long>(fv_cdiv((long)j1.rows * j1.Kpad, 256), 4096);
    if (d->dtype == FV_BF16)
      hipLaunchKernelGGL(weight_prep2_kernel<bf16>, dim3(j0.nb + j1.nb), dim3(256), 0, s, w_param, sigma, d->cout,
                         d->cin_valid, ks, j0, j1);
    else
      hipLaunchKernelGGL(weight_prep2_kernel<float>, dim3(j0.nb + j1.nb), dim3(256), 0, s, w_param, sigma, d->cout,
                         d->cin_valid, ks, j0, j1);
    return fv_check_launch("weight_prep2");
  }
  if (wk && use_c7n(d)) {
    hipLaunchKernelGGL(weight_prep_c7n_kernel, dim3(56), dim3(256), 0, s, w_param, sigma, (bf16*)wk, d->cout);
    if ((st = fv_check_launch("weight_prep_c7n"))) return st;
  } else if (wk && use_subpix_halo(d)) {
    const int nb = (int)std::min<long>(fv_cdiv(phase_wk_elems(d), 256), 4096);
    hipLaunchKernelGGL(weight_prep_phase_kernel<1>, dim3(nb), dim3(256), 0, s, w_param, sigma, (bf16*)wk,
                       4 * d->cout, 4 * (d->cin / 32), d->cout, d->cin_valid, 0);
    if ((st = fv_check_launch("weight_prep_phase1"))) return st;
  } else if (wk && use_subpix(d)) {
    const int rows = wrows(d->cout), Kp = kpad_of(2, d->cin);
    const long tot = 4L * rows * Kp;
    const int nb = (int)std::min<long>(fv_cdiv(tot, 256), 4096);
    hipLaunchKernelGGL(weight_prep_subpix_kernel<bf16>, dim3(nb), dim3(256), 0, s, w_param, sigma, (bf16*)wk, rows, Kp,
                       d->cout, d->cin_valid, fv_ilog2(d->cin));
    if ((st = fv_check_launch("weight_prep_subpix"))) return st;
  } else if (wk) {
    const int rows = wrows(d->cout), Kp = kpad_lay(smaj_wk(d), kpad_of(ks, d->cin));
    const long tot = (long)rows * Kp;
    const int nb = (int)std::min<long>(fv_cdiv(tot, 256), 4096);
    if (d->dtype == FV_BF16)
      hipLaunchKernelGGL(weight_prep_kernel<bf16>, dim3(nb), dim3(256), 0, s, w_param, sigma, (bf16*)wk,
                         rows, Kp, d->cout, d->cin_valid, fv_ilog2(d->cin), ks, ks * ks * d->cin, 0, smaj_wk(d));
    else
      hipLaunchKernelGGL(weight_prep_kernel<float>, dim3(nb), dim3(256), 0, s, w_param, sigma, (float*)wk,
                         rows, Kp, d->cout, d->cin_valid, fv_ilog2(d->cin), ks, ks * ks * d->cin, 0, 0);
    if ((st = fv_check_launch("weight_prep"))) return st;
  }
  if (wt && dgrad_halo_bn(d)) {
    const int nb = (int)std::min<long>(fv_cdiv(phase_wt_elems(d), 256), 4096);
    hipLaunchKernelGGL(weight_prep_phase_kernel<2>, dim3(nb), dim3(256), 0, s, w_param, sigma, (bf16*)wt, d->cin,
                       4 * (4 * d->cout / 32), d->cout, d->cin_valid, d->cout / 32);
    if ((st = fv_check_launch("weight_prep_phase2"))) return st;
  } else if (wt && use_dgrad_lowres(d)) {
    const int cin_t = pad_pow2_8(d->cout);
    const int rows = wrows(d->cin), Kp = 16 * cin_t;
    const long tot = (long)rows * Kp;
    const int nb = (int)std::min<long>(fv_cdiv(tot, 256), 4096);
    hipLaunchKernelGGL(weight_prep_s2_kernel<bf16>, dim3(nb), dim3(256), 0, s, w_param, sigma, (bf16*)wt, rows, Kp,
                       d->cout, d->cin_valid, fv_ilog2(cin_t));
    if ((st = fv_check_launch("weight_prep_s2"))) return st;
  } else if (wt) {
    const int cin_t = pad_pow2_8(d->cout);
    const int rows = wrows(d->cin), Kp = kpad_lay(smaj_wt(d), kpad_of(ks, cin_t));
    const long tot = (long)rows * Kp;
    const int nb = (int)std::min<long>(fv_cdiv(tot, 256), 4096);
    if (d->dtype == FV_BF16)
      hipLaunchKernelGGL(weight_prep_kernel<bf16>, dim3(nb), dim3(256), 0, s, w_param, sigma, (bf16*)wt,
                         rows, Kp, d->cout, d->cin_valid, fv_ilog2(cin_t), ks, ks * ks * cin_t, 1, smaj_wt(d));
    else
      hipLaunchKernelGGL(weight_prep_kernel<float>, dim3(nb), dim3(256), 0, s, w_param, sigma, (float*)wt,
                         rows, Kp, d->cout, d->cin_valid, fv_ilog2(cin_t), ks, ks * ks * cin_t, 1, 0);
    if ((st = fv_check_launch("weight_prep_t"))) return st;
  }
  return FV_OK;
}

int fv_conv_weight_prep_batchable(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  return !use_c7n(d) && !use_subpix(d) && !use_dgrad_lowres(d);
}

int fv_conv_weight_prep_multi(int n, const fv_conv_desc* descs, const float* const* w_params,
                              const float* const* sigmas, void* const* wks, void* const* wts, void* stream) {
  FV_REQUIRE(n >= 1 && n <= FV_WPREP_MAX && descs && w_params && sigmas && wks && wts, "weight_prep_multi: bad args");
  WPrepMulti m{};
  int nb_total = 0;
  const int dtype = descs[0].dtype;
  for (int i = 0; i < n; ++i) {
    const fv_conv_desc* d = &descs[i];
    int st = check_desc(d);
    if (st) return st;
    FV_REQUIRE(d->dtype == dtype, "weight_prep_multi: one dtype per call");
    FV_REQUIRE(fv_conv_weight_prep_batchable(d), "weight_prep_multi: conv %d needs a special layout", i);
    FV_REQUIRE(w_params[i] && wks[i], "weight_prep_multi: null pointer (conv %d)", i);
    const int ks = d->ksize;
    WPrepMJob j0{w_params[i], sigmas[i], wks[i], wrows(d->cout), kpad_lay(smaj_wk(d), kpad_of(ks, d->cin)),
                 fv_ilog2(d->cin),
                 ks * ks * d->cin, 0, 0, d->cout, d->cin_valid, ks, 0, smaj_wk(d)};
    j0.nb = (int)std::min<long>(fv_cdiv((long)j0.rows * j0.Kpad, 256), 256);
    nb_total = std::max(nb_total, j0.nb);
    m.j[m.n++] = j0;
    if (wts[i]) {
      const int cin_t = pad_pow2_8(d->cout);
      WPrepMJob j1{w_params[i], sigmas[i], wts[i], wrows(d->cin), kpad_lay(smaj_wt(d), kpad_of(ks, cin_t)),
                   fv_ilog2(cin_t),
                   ks * ks * cin_t, 1, 0, d->cout, d->cin_valid, ks, 0, smaj_wt(d)};
      j1.nb = (int)std::min<long>(fv_cdiv((long)j1.rows * j1.Kpad, 256), 256);
      nb_total = std::max(nb_total, j1.nb);
      m.j[m.n++] = j1;
    }
  }
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(weight_prep_multi_kernel<bf16>, dim3(nb_total, m.n), dim3(256), 0, s, m);
  else
    hipLaunchKernelGGL(weight_prep_multi_kernel<float>, dim3(nb_total, m.n), dim3(256), 0, s, m);
  return fv_check_launch("weight_prep_multi");
}

// store-pass record geometry (fv_store_reduce) of the launch `d` takes: records and pixels per
// record, 0 when that path has none.  The halo-staged 3x3 kernels only: 256-pixel tiles of 8
// waves (co tiles of 256 / 128) or 4 waves (co tiles of 64), one record per (tile, wave).
static int sr_geometry(const fv_conv_desc* d, int* bp) {
  if (d->dtype != FV_BF16 || use_c7n(d) || halo_tr(d) || use_subpix(d) || use_c64(d)) return 0;
  const int bn = halo3_bn(d);
  const long P = (long)d->n * d->h * d->w;
  if (!bn || d->cout % bn || P % 256) return 0;
  const int nw = bn == 64 ? 4 : 8;
  if (bp) *bp = 256 / nw;
  return (int)(P / 256 * nw);
}

extern "C++" {
// CUs of the current device (persistent grids), queried once
static int cu_count() {
  static int n = 0;
  if (!n) {
    int dev = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
        n <= 0)
      n = 256;
  }
  return n;
}
// persistent tiles for conv3_halo_fwd3 (PERS); FV_PERS=0 launches one block per tile (A/B).
// Read per call.
static bool pers_on() {
  const char* e = getenv("FV_PERS");
  return !(e && e[0] == '0');
}
// one conv3_halo_fwd3 launch over ntiles tiles: schedule SCH 2 (stagger) unless FV_RES_SCHED
// says 0 / 1 (-> 0), persistent (one block per CU) when there are more tiles than CUs
template <int WN, int WM, int RN, int RM, int NSB, int MODE>
static void launch_h3(int ntiles, hipStream_t s, const ConvArgs& a, unsigned xb) {
  const int sch = res_sched(2) >= 2 ? 2 : 0;
  // FV_PERS_GRID=k caps the persistent grid at k blocks (tests: several tiles per block at
  // small shapes)
  const char* e = getenv("FV_PERS_GRID");
  const int cap = (e && atoi(e) > 0) ? atoi(e) : cu_count();
  // (the 256-row co tiles spill ~130 registers in the persistent form -- the epilogue's
  // read-back beside the carried tile state -- and ran res fwd 120 -> 166 us, r5; kept to the
  // smaller co tiles: AFE.down1's data gradient 366 -> 348 us)
  const bool pers = WN * RN * 16 < 256 && pers_on() && ntiles > cap;
  const dim3 g(pers ? cap : ntiles), b(64 * WN * WM);
  if constexpr (WN * RN * 16 < 256) {
    if (pers) {
      if (sch == 2) hipLaunchKernelGGL((conv3_halo_fwd3<WN, WM, RN, RM, NSB, 2, MODE, true>), g, b, 0, s, a, xb, ntiles);
      else hipLaunchKernelGGL((conv3_halo_fwd3<WN, WM, RN, RM, NSB, 0, MODE, true>), g, b, 0, s, a, xb, ntiles);
      return;
    }
  }
  {
    if (sch == 2) hipLaunchKernelGGL((conv3_halo_fwd3<WN, WM, RN, RM, NSB, 2, MODE, false>), g, b, 0, s, a, xb, ntiles);
    else hipLaunchKernelGGL((conv3_halo_fwd3<WN, WM, RN, RM, NSB, 0, MODE, false>), g, b, 0, s, a, xb, ntiles);
  }
}
}  // extern "C++"

// 1x1 convs with K = 256 / 512 input channels and whole 256-channel output groups (the mid
// convs and their data gradients) on the pixel-stream kernel conv1x1_stream; FV_C1S=0 keeps
// conv_fwd_v2 (A/B).  Read per call.
static bool use_c1s(const fv_conv_desc* d) {
  const char* e = getenv("FV_C1S");
  if (e && e[0] == '0') return false;
  if (!use_v2(d) || d->ksize != 1 || d->upsample || d->pro_act) return false;
  if ((d->cin != 256 && d->cin != 512) || d->cout % 256 || d->ldy != d->cout) return false;
  const long P = (long)d->n * d->h * d->w;
  return P % (32768 / d->cin) == 0 && P * d->cout * 2 < (1L << 31);   // (both tile sizes)
}

static int conv_run(const fv_conv_desc* d, const void* x, const void* wk, const float* bias,
                    const float* psc, const float* psh, const void* res, void* y, float* stats,
                    hipStream_t s, const fv_store_reduce* sr = nullptr) {
  ConvArgs a{};
  if (sr && sr->mode) {
    FV_REQUIRE(sr_geometry(d, nullptr) > 0, "store-pass records not available for this conv (query fv_conv2d_sr_records)");
    FV_REQUIRE(sr->records, "store-pass records: null buffer");
    FV_REQUIRE(sr->mode == 1 || (sr->mode == 2 && sr->bn_input && sr->mean && sr->invstd && sr->gamma && sr->beta && !res),
               "store-pass records: bad mode / BN arguments");
    FV_REQUIRE(!stats, "store-pass records and accumulator statistics in one call are not supported");
    a.spm = sr->mode;
    a.sprec = sr->records;
    a.bnm = sr->mean; a.bni = sr->invstd; a.bng = sr->gamma; a.bnb = sr->beta; a.bns = sr->slope;
    if (sr->mode == 2) res = sr->bn_input;        // prefetched as a residual, not added
  }
  const FwdTile t = fwd_tile(d->cout);
  a.x = x; a.w = wk; a.bias = bias; a.psc = psc; a.psh = psh; a.slope = d->pro_slope;
  a.res = res; a.y = y; a.stats = stats;
  a.nrec = stats ? fv_conv2d_stats_blocks(d) : 0;
  a.N = d->n; a.H = d->h; a.W = d->w;
  a.Hin = d->upsample ? d->h / 2 : d->h;
  a.Win = d->upsample ? d->w / 2 : d->w;
  a.P = d->n * d->h * d->w;
  a.Cin = d->cin; a.lgCin = fv_ilog2(d->cin);
  a.Cout = d->cout; a.ldy = d->ldy;
  a.K = d->ksize * d->ksize * d->cin; a.Kpad = kpad_of(d->ksize, d->cin); a.nks = a.Kpad / BK;
  a.sigmoid = d->epi_sigmoid; a.nchw = d->out_nchw_f32;
  a.ntn = fv_cdiv(d->cout, t.bn);
  int st;
  // the weight image the caller sized with fv_conv_wk_elems(d) (fv_conv_wt_elems for a data
  // gradient: the same function of the transposed descriptor) must hold every row and k this
  // launch's weight DMA reads: rows = the co tiles it covers, k = its K per row (r4 fault: a
  // tile larger than the image read past its end)
  const long wk_have = (long)fv_conv_wk_elems(d);
  auto wext = [&](long rows, long kk, const char* what) {
    if (rows * kk > wk_have) {
      fv_set_error("conv %s: weight DMA extent %ld x %ld > weight image %ld elements", what, rows, kk, wk_have);
      return FV_E_BADARG;
    }
    return FV_OK;
  };
  if (use_c7n(d)) {
    FV_REQUIRE(!res, "out_conv kernel: no residual");
    const unsigned xb = (unsigned)((long)d->n * d->h * d->w * 64 * 2);
    const int band = c7n_band(d);
    const int nblk = d->n * (d->h / band) * (d->w / 64);
    hipLaunchKernelGGL(conv7_n3_fwd2, dim3(nblk), dim3(512), 0, s, a, xb, band);
    return fv_check_launch("conv2d_fwd_c7n2");
  }
  // the 64-channel band kernel has no residual / store-pass epilogue: such a launch (a 64-channel
  // ResBlock conv) runs conv_fwd_v2, which reads the same plain [co][Kpad] weights (lay_of)
  const bool c64 = use_c64(d);
  if (c64 && !res && !a.spm) {
    if ((st = wext(d->cout, kpad_of(3, 64), "c64"))) return st;
    const int nb = c64_bands(d);
    const int nblk = d->n * (d->w / 64) * (d->cout / 64) * nb;
    const unsigned xb = (unsigned)((long)d->n * d->h * d->w * 64 * 2);
    hipLaunchKernelGGL(conv3c64_fwd, dim3(nblk), dim3(512), 0, s, a, xb, nb);
    return fv_check_launch("conv2d_fwd_c64");
  }
  if (use_c74(d)) {
    FV_REQUIRE(!res, "packed 7x7 conv: no residual");
    const int ntiles = d->n * (d->h / C74_TR) * (d->w / 64);
    const unsigned xb = (unsigned)((long)d->n * d->h * d->w * d->cin * 2);
    FV_REQUIRE(!a.stats || a.nrec == c74_grid(d), "packed 7x7 conv: %d BN records for %d blocks", a.nrec, c74_grid(d));
    hipLaunchKernelGGL(conv7c4_fwd, dim3(c74_grid(d)), dim3(512), 0, s, a, xb, ntiles);
    return fv_check_launch("conv2d_fwd_c74");
  }
  if (const int tr = halo_tr(d)) {
    if ((st = wext(plan_tile(d).bn, kpad_of(7, d->cin), "halo7"))) return st;
    a.lgtw = 6;
    const int nblk = d->n * (d->h / tr) * (d->w / 64);
    const unsigned xb = (unsigned)((long)d->n * d->h * d->w * d->cin * 2);
    if (d->cin == 8)
      hipLaunchKernelGGL((conv_halo_fwd<7, 8, 4, 4, true, false>), dim3(nblk), dim3(512), 0, s, a, xb);
    else
      hipLaunchKernelGGL((conv_halo_fwd<7, 64, 1, 2, false, true>), dim3(nblk), dim3(512), 0, s, a, xb);
    return fv_check_launch("conv2d_fwd_halo");
  }
  if (use_upband(d)) {
    FV_REQUIRE(!res && !a.spm, "sub-pixel band conv: no residual / store-pass records");
    a.Ho = d->h; a.Wo = d->w;
    a.Kpad = kpad_of(2, d->cin);
    a.wphase = wrows(d->cout) * a.Kpad;
    if ((st = wext(4L * wrows(d->cout), a.Kpad, "upband"))) return st;
    const int hl = d->h / 2, wl = d->w / 2;
    const long base = (long)d->n * (wl / 32) * (d->cout / 64);
    int nb = 1;
    while (base * nb < 256 && hl % (nb * 16) == 0) nb *= 2;      // bands of a multiple of 8 rows
    const int nblk = (int)(base * nb);
    const unsigned xb = (unsigned)((long)d->n * hl * wl * 128 * 2);
    hipLaunchKernelGGL(conv3up_band_fwd, dim3(nblk), dim3(512), 0, s, a, xb, nb);
    return fv_check_launch("conv2d_fwd_upband");
  }
  if (use_subpix_halo(d)) {
    FV_REQUIRE(!res && !a.spm, "sub-pixel conv: no residual / store-pass records");
    a.H = a.Hin; a.W = a.Win;                       // tile space = the low-res input image
    a.Ho = d->h; a.Wo = d->w;
    a.P = d->n * a.H * a.W;
    a.lgtw = 6;
    a.wus = 4 * d->cout * 64;                       // one unit = 4 phases x cout rows of 64 B
    a.ntn = d->cout / 64;
    const int nblk = a.ntn * d->n * (a.H / 4) * (a.W / 64);
    const unsigned xb = (unsigned)((long)d->n * a.H * a.W * d->cin * 2);
    // the weight DMA of the last unit ends inside the image the queries size
    FV_REQUIRE((long)4 * (d->cin / 32) * a.wus / 2 <= phase_wk_elems(d), "sub-pixel halo conv: weight image");
    launch_h3<4, 2, 4, 8, 2, 1>(nblk, s, a, xb);
    return fv_check_launch("conv2d_fwd_subpix_halo");
  }
  if (use_subpix(d)) {
    FV_REQUIRE(!res, "sub-pixel conv: no residual");
    const FwdTile t2 = fwd_tile_v2(d->cout);
    a.H = a.Hin; a.W = a.Win;                       // tile space = the low-res input image
    a.Ho = d->h; a.Wo = d->w;
    a.P = d->n * a.H * a.W;
    a.lgw = fv_ilog2(a.W); a.lghw = fv_ilog2(a.H * a.W);
    a.Kpad = kpad_of(2, d->cin);
    a.nks = a.Kpad / BK2;
    a.ntn = fv_cdiv(d->cout, t2.bn);
    a.wphase = wrows(d->cout) * a.Kpad;
    if ((st = wext(4L * a.ntn * t2.bn, a.Kpad, "subpix"))) return st;
    const int nblk2 = 4 * a.ntn * (a.P / t2.bm);
    const long xb = (long)d->n * a.Hin * a.Win * d->cin * 2;
    st = launch_v2(a, 2, t2, 2, nblk2, (unsigned)xb, s);
    if (st) {
      fv_set_error("sub-pixel conv variant unsupported (cout=%d)", d->cout);
      return st;
    }
    return fv_check_launch("conv2d_fwd_subpix");
  }
  if (const int bn = c64 ? 0 : halo3_bn(d)) {
    FV_REQUIRE(!(res && stats), "conv v2: residual and BN statistics in one call are not supported");
    a.lgtw = 6;
    a.wus = wk_rows(d) * 64;
    a.ntn = d->cout / bn;
    // stage-major: units of wk_rows(d) rows x 32; the tiles read rows [0, ntn * bn) of each
    if ((st = wext(a.ntn * bn, 9L * d->cin, "halo3")) || (st = wext(wk_rows(d), 9L * d->cin, "halo3 units")))
      return st;
    const int nblk = a.ntn * d->n * (d->h / 4) * (d->w / 64);
    const unsigned xb = (unsigned)((long)d->n * d->h * d->w * d->cin * 2);
    // linear-halo pair-of-taps kernel (conv3_halo_fwd3) for the 256 / 128-channel co tiles;
    // conv3_halo_fwd2 (XOR-swizzled halo) for 64-channel co tiles (AFE.down1's data gradient:
    // 448 us against 667 us on fwd3) and channel counts that are not a multiple of 64.
    // (measured and not kept, r2: the single-tap halo loop -- down2 dgrad 369 vs 324 us,
    // down1 dgrad 433 vs 414 us; a 3-deep weight ring for the 256-channel tiles, 2.5 % slower;
    // 8-row tiles for the 64-channel co tile, 418 -> 420 us; weight-DMA pieces spread between
    // the MFMA rows as conv_wgrad_v2 does, res conv forward 134 -> 160 us.  r3, res conv forward
    // in alternating runs on one box: halo chunks issued after the weight stage and left in
    // flight one step longer 126 -> 133 us; a ping-pong schedule (waves 4-7 one phase behind,
    // each wave's fragment reads + DMA issue beside its SIMD partner's MFMAs, 3-stage ring,
    // 2 barriers per step) 134 -> 142 us; 128 co x 512 px tiles, 25 instead of 40 KB of LDS-DMA
    // per step, 153 -> 157 (fwd2) / 161 us (ping-pong).  The clock-stamp build (build.py --diag)
    // puts the step at ~3400 cycles against 2048 of MFMA issue; with the MFMAs removed the
    // ping-pong loop still took 92 % of its time, with the fragment reads removed 65 %.
    // Stage-major weights (every DMA piece one contiguous KB, weight_prep_body smaj): res
    // fwd / dgrad 127 / 121.5 -> 122 / 117 us, down2 dgrad 317 -> 301 us (kept).  The weights
    // off the LDS-DMA path -- each wave's A fragments loaded to registers two / one taps ahead,
    // the halo register-staged, one barrier per 32-channel chunk: 126 -> 134 us (not kept).
    // r4: the 256 x 256 tile on 4 waves of 128 co x 128 px (one wave per SIMD, 512 registers,
    // a third fewer LDS fragment bytes per MFMA): res fwd / dgrad 133 / 127 -> 162 / 153 us,
    // the SIMD partner's MFMAs no longer cover a wave's fragment reads and barrier waits.  The B
    // fragments of the column-shifted taps (s = 1, 2) made from the previous tap's in registers
    // by DPP lane shifts (row_shl:1 | row_shr:15 of the next fragment, the row-end pixel read
    // as a broadcast: 2 instead of 8 B reads per tap): res fwd / dgrad 132-135 / 125-128 ->
    // 136-138 / 131-132 us, step +0.14 ms.  The weight stages after the first two through
    // registers (buffer_load_dwordx4 a step ahead, ds_write_b128 after the next barrier) instead
    // of LDS-DMA: res fwd / dgrad 147 / 136 -> 150.5 / 141 us, Generator.in_conv 147-152 ->
    // 160-162 us, step +0.17 ms.)
    if (bn >= 128 && a.Cin % 64 == 0) {
      if (bn == 256) launch_h3<4, 2, 4, 8, 2, 0>(nblk, s, a, xb);
      else launch_h3<2, 4, 4, 4, 3, 0>(nblk, s, a, xb);
    } else if (bn == 256) {
      hipLaunchKernelGGL((conv3_halo_fwd2<4, 2, 4, 8, 2>), dim3(nblk), dim3(512), 0, s, a, xb);
    } else if (bn == 128) {
      hipLaunchKernelGGL((conv3_halo_fwd2<2, 4, 4, 4, 3>), dim3(nblk), dim3(512), 0, s, a, xb);
    } else if (d->h % 8 == 0 && a.Cin % 64 == 0 && c64t_on()) {
      // 64-channel co tile (AFE.down1's data gradient): 8 waves over 8 rows x 64 px, the
      // linear-halo kernel (fwd2's XOR-swizzled halo addressing was its VALU
      // limiter); waves 0-3 issue the 4 weight pieces of a tap
      const int nblk8 = a.ntn * d->n * (d->h / 8) * (d->w / 64);
      launch_h3<1, 8, 4, 4, 2, 0>(nblk8, s, a, xb);
    } else {
      hipLaunchKernelGGL((conv3_halo_fwd2<1, 4, 4, 4, 3>), dim3(nblk), dim3(256), 0, s, a, xb);
    }
    return fv_check_launch("conv2d_fwd_halo3");
  }
  if (use_c1s(d) && !res && !stats && !a.spm) {
    if ((st = wext(d->cout, a.Kpad, "c1s"))) return st;
    FV_REQUIRE(a.Kpad == d->cin, "1x1 stream conv: K %d != Kpad %d", d->cin, a.Kpad);
    const int ncg = d->cout / 256;
    const int grid = std::max(8 * ncg, cu_count() / (8 * ncg) * (8 * ncg));
    const unsigned xb = (unsigned)((long)a.P * d->cin * 2);
    // FV_C1S_BP=64 / 128: pixels per tile for K = 256 (halved for K = 512): 4 slots of 32 KB
    // or 2 of 64 KB (A/B; read per call)
    const char* e = getenv("FV_C1S_BP");
    const bool big = e && atoi(e) == 128;
    if (d->cin == 256) {
      if (big) hipLaunchKernelGGL((conv1x1_stream<256, 128>), dim3(grid), dim3(512), 0, s, a, xb);
      else hipLaunchKernelGGL((conv1x1_stream<256, 64>), dim3(grid), dim3(512), 0, s, a, xb);
    } else {
      if (big) hipLaunchKernelGGL((conv1x1_stream<512, 64>), dim3(grid), dim3(512), 0, s, a, xb);
      else hipLaunchKernelGGL((conv1x1_stream<512, 32>), dim3(grid), dim3(512), 0, s, a, xb);
    }
    return fv_check_launch("conv2d_fwd_c1s");
  }
  if (use_v2(d)) {
    FV_REQUIRE(!(res && stats), "conv v2: residual and BN statistics in one call are not supported");
    const FwdTile t2 = fwd_tile_v2(d->cout);
    a.ntn = fv_cdiv(d->cout, t2.bn);
    a.nks = a.Kpad / BK2;            // 64-deep steps; the 32-deep kernels double it themselves
    if ((st = wext((long)a.ntn * t2.bn, a.Kpad, "v2"))) return st;
    const int nblk2 = a.ntn * fv_cdiv(a.P, t2.bm);
    const long xb = (long)d->n * a.Hin * a.Win * d->cin * 2;
    st = launch_v2(a, d->ksize, t2, d->upsample, nblk2, (unsigned)xb, s);
    if (st) {
      fv_set_error("conv v2 variant unsupported (k=%d ups=%d)", d->ksize, d->upsample);
      return st;
    }
    return fv_check_launch("conv2d_fwd_v2");
  }
  const int nblk = a.ntn * fv_cdiv(a.P, t.bm);
  if ((st = wext((long)a.ntn * t.bn, a.Kpad, "v1"))) return st;
  st = d->dtype == FV_BF16 ? launch_fwd<bf16>(a, d->ksize, t, d->pro_act, d->upsample, nblk, s)
                           : launch_fwd<float>(a, d->ksize, t, d->pro_act, d->upsample, nblk, s);
  if (st) {
    fv_set_error("conv variant unsupported (k=%d pro=%d ups=%d)", d->ksize, d->pro_act, d->upsample);
    return st;
  }
  return fv_check_launch("conv2d_fwd");
}

#ifdef FV_DIAG
// diagnostic build: copy the stamp table (g_diag) to the host
int fv_diag_read(unsigned long long* host, int n) {
  const int cap = (int)(sizeof(g_diag) / sizeof(g_diag[0]));
  if (n > cap) n = cap;
  if (hipDeviceSynchronize() != hipSuccess) return 1;
  return hipMemcpyFromSymbol(host, HIP_SYMBOL(g_diag), (size_t)n * sizeof(unsigned long long)) == hipSuccess ? 0 : 1;
}
int fv_diag_clear(void) {
  void* p = nullptr;
  if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_diag)) != hipSuccess) return 1;
  return hipMemset(p, 0, sizeof(g_diag)) == hipSuccess ? 0 : 1;
}
#endif

int fv_conv2d_fwd(const fv_conv_desc* d, const void* x, const void* wk, const float* bias,
                  const float* pro_scale, const float* pro_shift, const void* res, void* y,
                  float* stats, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(x && wk && y, "null pointer");
  FV_REQUIRE(!d->pro_act || (pro_scale && pro_shift), "prologue needs scale/shift");
  FV_REQUIRE(d->out_nchw_f32 || d->ldy >= d->cout, "ldy < cout");
  FV_REQUIRE(!res || d->ldy % 4 == 0, "residual needs ldy % 4 == 0");
  FV_REQUIRE(d->out_nchw_f32 || d->cout % 4 == 0 || d->ldy >= d->cout, "bad ldy");
  return conv_run(d, x, wk, bias, pro_scale, pro_shift, res, y, stats, (hipStream_t)stream);
}

// the forward-conv descriptor the data gradient of `d` runs as (transposed, flipped weights)
static fv_conv_desc dgrad_desc(const fv_conv_desc* d) {
  fv_conv_desc t{};
  t.dtype = d->dtype;
  t.n = d->n; t.h = d->h; t.w = d->w;
  t.cin = pad_pow2_8(d->cout);
  t.cin_valid = d->cout;
  t.cout = d->cin;   // every (padded) input channel; padded ones come out 0
  t.ldy = d->cin;
  t.ksize = d->ksize;
  return t;
}

int fv_conv2d_sr_records(const fv_conv_desc* d, int dgrad, int* record_pixels) {
  if (check_desc(d) != FV_OK) return 0;
  if (dgrad) {
    if (d->upsample) return 0;
    const fv_conv_desc t = dgrad_desc(d);
    return sr_geometry(&t, record_pixels);
  }
  return sr_geometry(d, record_pixels);
}

int fv_conv2d_fwd_sr(const fv_conv_desc* d, const void* x, const void* wk, const float* bias, const void* res, void* y,
                     const fv_store_reduce* sr, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(x && wk && y && sr && sr->mode == 1, "fwd_sr: null pointer or mode != 1");
  FV_REQUIRE(!d->pro_act && !d->out_nchw_f32 && d->ldy == d->cout, "fwd_sr: plain NHWC output only");
  return conv_run(d, x, wk, bias, nullptr, nullptr, res, y, nullptr, (hipStream_t)stream, sr);
}

int fv_conv2d_bwd_data_sr(const fv_conv_desc* d, const void* dy, int ldy_dy, const void* wt, void* dx,
                          const fv_store_reduce* sr, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(dy && wt && dx && sr && sr->mode == 2 && !d->upsample, "bwd_data_sr: bad argument");
  const fv_conv_desc t = dgrad_desc(d);
  FV_REQUIRE(ldy_dy == t.cin, "bwd_data: dy channel stride must be %d (got %d)", t.cin, ldy_dy);
  return conv_run(&t, dy, wt, nullptr, nullptr, nullptr, nullptr, dx, nullptr, (hipStream_t)stream, sr);
}

int fv_conv2d_bwd_data(const fv_conv_desc* d, const void* dy, int ldy_dy, const void* wt, void* dx,
                       void* stream) {
  int st = check_desc(d);
  if (st) return st;
  const fv_conv_desc t = dgrad_desc(d);
  FV_REQUIRE(ldy_dy == t.cin, "bwd_data: dy channel stride must be %d (got %d)", t.cin, ldy_dy);
  if (const int bn = dgrad_halo_bn(d)) {
    FV_REQUIRE(dy && wt && dx, "null pointer");
    ConvArgs a{};
    a.x = dy; a.w = wt; a.y = dx;
    a.N = d->n; a.H = d->h / 2; a.W = d->w / 2; a.Hin = d->h; a.Win = d->w;
    a.Ho = a.H; a.Wo = a.W;
    a.P = d->n * a.H * a.W;
    a.Cin = 4 * d->cout;                            // the 4 phase planes of dy as input channels
    a.K = d->cout;                                  // dy's channel stride
    a.Cout = d->cin; a.ldy = d->cin;
    a.lgtw = 6;
    a.wus = d->cin * 64;
    a.ntn = d->cin / bn;
    const int nblk = a.ntn * d->n * (a.H / 4) * (a.W / 64);
    const unsigned xb = (unsigned)((long)d->n * d->h * d->w * d->cout * 2);
    FV_REQUIRE((long)(a.Cin / 32) * 4 * a.wus / 2 <= phase_wt_elems(d), "low-res halo dgrad: weight image");
    if (bn == 256) launch_h3<4, 2, 4, 8, 2, 2>(nblk, (hipStream_t)stream, a, xb);
    else launch_h3<2, 4, 4, 4, 3, 2>(nblk, (hipStream_t)stream, a, xb);
    return fv_check_launch("conv2d_bwd_data_lowres_halo");
  }
  if (use_dgrad_lowres(d)) {
    FV_REQUIRE(dy && wt && dx, "null pointer");
    ConvArgs a{};
    const FwdTile t2 = fwd_tile_v2(d->cin);
    a.x = dy; a.w = wt; a.y = dx;
    a.N = d->n; a.H = d->h / 2; a.W = d->w / 2; a.Hin = d->h; a.Win = d->w;
    a.Ho = a.H; a.Wo = a.W;
    a.P = d->n * a.H * a.W;
    a.Cin = t.cin; a.lgCin = fv_ilog2(t.cin);
    a.Cout = d->cin; a.ldy = d->cin;
    a.Kpad = 16 * t.cin; a.K = a.Kpad; a.nks = a.Kpad / BK2;
    a.ntn = fv_cdiv(d->cin, t2.bn);
    const int nblk = a.ntn * fv_cdiv(a.P, t2.bm);
    const long xb = (long)d->n * d->h * d->w * t.cin * 2;
    const int st = launch_v2(a, 4, t2, 3, nblk, (unsigned)xb, (hipStream_t)stream);
    if (st) {
      fv_set_error("low-res dgrad variant unsupported (cin=%d)", d->cin);
      return st;
    }
    return fv_check_launch("conv2d_bwd_data_lowres");
  }
  return conv_run(&t, dy, wt, nullptr, nullptr, nullptr, nullptr, dx, nullptr, (hipStream_t)stream);
}

int fv_conv2d_wgrad_nsplit(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  return plan_wgrad(d).nsplit;
}

size_t fv_conv2d_wgrad_slab_elems(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  const WgPlan p = plan_wgrad(d);
  return (size_t)(p.sub ? 4 : 1) * p.nsplit * p.CW * p.KW;
}

size_t fv_conv2d_wgrad_bias_slab_elems(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  const WgPlan p = plan_wgrad(d);
  return (size_t)(p.sub ? 4 : 1) * p.nsplit * p.CW;
}

int fv_conv2d_bwd_weight(const fv_conv_desc* d, const void* x, const float* pro_scale,
                         const float* pro_shift, const void* dy, int ldy_dy, float* slab,
                         float* bias_slab, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(x && dy && slab, "null pointer");
  FV_REQUIRE(ldy_dy % 8 == 0 && ldy_dy >= d->cout, "wgrad: dy channel stride must be a multiple of 8 >= cout");
  FV_REQUIRE(!d->pro_act || (pro_scale && pro_shift), "prologue needs scale/shift");
  const WgPlan t = plan_wgrad(d);
  const int Hin = d->upsample ? d->h / 2 : d->h, Win = d->upsample ? d->w / 2 : d->w;
  const long P = (long)d->n * d->h * d->w;
  if (t.v2 == 5) {
    FV_REQUIRE(P * ldy_dy * 2 < (1L << 31) && P * d->cin * 2 < (1L << 31), "wgrad: operand larger than 2 GB");
    H3Wg2Args a{};
    a.x = x; a.dy = dy; a.slab = slab; a.bslab = bias_slab;
    a.H = d->h; a.W = d->w; a.Cout = d->cout; a.ldd = ldy_dy;
    a.nseg = t.nsteps; a.rows = t.sps; a.nct = t.ntc;
    a.ldx = d->cin; a.nci = t.ntk;
    a.xbytes = (unsigned)(P * d->cin * 2);
    a.dybytes = (unsigned)(P * ldy_dy * 2);
    hipLaunchKernelGGL(conv3_halo_wgrad2<4>, dim3(t.ntc * t.ntk * t.nsplit), dim3(512), 0, (hipStream_t)stream, a);
    return fv_check_launch("conv2d_bwd_weight_halo3s");
  }
  if (t.v2 == 6) {
    FV_REQUIRE(P * ldy_dy * 2 < (1L << 31) && (long)d->n * Hin * Win * d->cin * 2 < (1L << 31),
               "wgrad: operand larger than 2 GB");
    UpWgArgs a{};
    a.x = x; a.dy = dy; a.slab = slab; a.bslab = bias_slab;
    a.Hin = Hin; a.Win = Win; a.Cout = d->cout; a.Cin = d->cin; a.ldd = ldy_dy;
    a.nct = t.ntc; a.nci = t.ntk; a.units = t.nsteps; a.spb = t.sps; a.nsplit = t.nsplit;
    a.xbytes = (unsigned)((long)d->n * Hin * Win * d->cin * 2);
    a.dybytes = (unsigned)(P * ldy_dy * 2);
    hipLaunchKernelGGL(conv3_up_wgrad<2>, dim3(t.ntc * t.ntk * t.nsplit), dim3(512), 0, (hipStream_t)stream, a);
    return fv_check_launch("conv2d_bwd_weight_up");
  }
  if (t.v2 == 3) {
    FV_REQUIRE(ldy_dy == 8, "wgrad (out_conv 7x7): dy channel stride must be 8 (got %d)", ldy_dy);
    W7Args a{};
    a.x = x; a.dy = dy; a.slab = slab; a.bslab = bias_slab;
    a.H = d->h; a.W = d->w; a.ldd = ldy_dy; a.cout = d->cout;
    a.seg_rows = t.sps; a.nseg = t.nsteps;
    a.xbytes = (unsigned)(P * 64 * 2);
    a.dybytes = (unsigned)(P * 8 * 2);
    hipLaunchKernelGGL(conv7_n3_wgrad, dim3(t.nsplit), dim3(512), 0, (hipStream_t)stream, a);
    return fv_check_launch("conv2d_bwd_weight_c7");
  }
  if (t.v2 == 2) {
    const int ldd_need = d->cin == 8 ? 64 : 8;
    FV_REQUIRE(ldy_dy == ldd_need, "wgrad (7x7 halo): dy channel stride must be %d (got %d)", ldd_need, ldy_dy);
    HaloWgArgs a{};
    a.x = x; a.dy = dy; a.slab = slab; a.bslab = bias_slab;
    a.H = d->h; a.W = d->w; a.ldd = ldy_dy; a.K = d->ksize * d->ksize * d->cin;
    a.KW = t.KW; a.CW = t.CW; a.ntiles = t.nsteps; a.cout = d->cout;
    a.xbytes = (unsigned)(P * d->cin * 2);
    a.dybytes = (unsigned)(P * ldy_dy * 2);
    FV_REQUIRE(t.KW == (halo_wg_pk(d) ? 224 : fv_cdiv(a.K, 16) * 16), "7x7 halo wgrad: slab row length");
    if (d->cin == 8 && halo_wg_pk(d))
      hipLaunchKernelGGL((conv_halo_wgrad<7, 8, 4, 4, true>), dim3(t.nsplit), dim3(512), 0, (hipStream_t)stream, a);
    else if (d->cin == 8)
      hipLaunchKernelGGL((conv_halo_wgrad<7, 8, 4, 4>), dim3(t.nsplit), dim3(512), 0, (hipStream_t)stream, a);
    else
      hipLaunchKernelGGL((conv_halo_wgrad<7, 64, 1, 2>), dim3(t.nsplit), dim3(512), 0, (hipStream_t)stream, a);
    return fv_check_launch("conv2d_bwd_weight_halo");
  }
  if (t.sub) {
    FV_REQUIRE(P * ldy_dy * 2 < (1L << 31), "wgrad: dy larger than 2 GB");
    Wg2Args a{};
    a.x = x; a.dy = dy; a.slab = slab; a.bslab = bias_slab;
    a.H = Hin; a.W = Win; a.Hin = Hin; a.Win = Win; a.P = d->n * Hin * Win;
    a.Ho = d->h; a.Wo = d->w; a.nsplit = t.nsplit;
    a.lgCin = fv_ilog2(d->cin);
    a.K = 4 * d->cin;
    a.KW = t.KW; a.ldd = ldy_dy; a.CW = t.CW;
    a.ntk = t.ntk; a.ntc = t.ntc; a.nsteps = t.nsteps; a.sps = t.sps;
    a.fhw = make_fastdiv((uint32_t)(Hin * Win));
    a.fw = make_fastdiv((uint32_t)Win);
    a.fh = make_fastdiv((uint32_t)Hin);
    a.rowal = 1;
    a.il = 1;
    a.xbytes = (unsigned)((long)d->n * Hin * Win * d->cin * 2);
    a.dybytes = (unsigned)(P * ldy_dy * 2);
    const int nblk = 4 * t.ntk * t.ntc * t.nsplit;
    st = launch_wg2(a, 2, t, 0, nblk, (hipStream_t)stream);
    if (st) {
      fv_set_error("sub-pixel wgrad variant unsupported (cfg %d)", t.cfg);
      return st;
    }
    return fv_check_launch("conv2d_bwd_weight_subpix");
  }
  if (t.v2) {
    FV_REQUIRE(P * ldy_dy * 2 < (1L << 31), "wgrad: dy larger than 2 GB");
    Wg2Args a{};
    a.x = x; a.dy = dy; a.slab = slab; a.bslab = bias_slab;
    a.H = d->h; a.W = d->w; a.Hin = Hin; a.Win = Win; a.P = (int)P;
    a.lgCin = fv_ilog2(d->cin);
    a.K = d->ksize * d->ksize * d->cin;
    a.KW = t.KW; a.ldd = ldy_dy; a.CW = t.CW;
    a.ntk = t.ntk; a.ntc = t.ntc; a.nsteps = t.nsteps; a.sps = t.sps;
    a.fhw = make_fastdiv((uint32_t)(d->h * d->w));
    a.fw = make_fastdiv((uint32_t)d->w);
    a.fh = make_fastdiv((uint32_t)d->h);
    a.rowal = (d->w % t.px) == 0;
    a.il = 1;
    a.xbytes = (unsigned)((long)d->n * Hin * Win * d->cin * 2);
    a.dybytes = (unsigned)(P * ldy_dy * 2);
    const int nblk = t.ntk * t.ntc * t.nsplit;
    st = launch_wg2(a, d->ksize, t, d->upsample, nblk, (hipStream_t)stream);
    if (st) {
      fv_set_error("wgrad v2 variant unsupported (k=%d ups=%d bkt=%d bc=%d)", d->ksize, d->upsample, t.bkt, t.bc);
      return st;
    }
    return fv_check_launch("conv2d_bwd_weight_v2");
  }
  WgArgs a{};
  a.x = x; a.psc = pro_scale; a.psh = pro_shift; a.slope = d->pro_slope;
  a.dy = dy; a.slab = slab; a.bslab = bias_slab;
  a.N = d->n; a.H = d->h; a.W = d->w;
  a.Hin = Hin;
  a.Win = Win;
  a.P = (int)P;
  a.Cin = d->cin; a.lgCin = fv_ilog2(d->cin);
  a.K = d->ksize * d->ksize * d->cin;
  a.ntk = t.ntk; a.KW = t.KW;
  a.Cout = d->cout; a.ldd = ldy_dy;
  a.ntc = t.ntc; a.CW = t.CW;
  a.nsteps = t.nsteps;
  a.steps_per_split = t.sps;
  const int nblk = t.ntk * t.ntc * t.nsplit;
  st = d->dtype == FV_BF16 ? launch_wg<bf16>(a, d->ksize, t, d->pro_act, d->upsample, nblk, (hipStream_t)stream)
                           : launch_wg<float>(a, d->ksize, t, d->pro_act, d->upsample, nblk, (hipStream_t)stream);
  if (st) {
    fv_set_error("wgrad variant unsupported (k=%d pro=%d ups=%d)", d->ksize, d->pro_act, d->upsample);
    return st;
  }
  return fv_check_launch("conv2d_bwd_weight");
}

int fv_conv2d_wgrad_reduce(const fv_conv_desc* d, const float* slab, const float* bias_slab,
                           float* dw_param, float* db, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(slab && dw_param, "null pointer");
  FV_REQUIRE(!db || bias_slab, "db needs the bias slab");
  const WgPlan t = plan_wgrad(d);
  if (t.v2 == 3) {
    // the two passes reuse the slab rows in place (the slabs are dead after the reduce)
    const int ncol = W7_COLS + (db ? 4 : 0);
    const int G = t.nsplit >= 256 ? 16 : (t.nsplit >= 16 ? 4 : 1);
    const int rpg = fv_cdiv(t.nsplit, G);
    hipLaunchKernelGGL(w7_reduce1_kernel, dim3(fv_cdiv(ncol, 64), G), dim3(256), 0, (hipStream_t)stream,
                       const_cast<float*>(slab), const_cast<float*>(bias_slab), t.nsplit, rpg, ncol);
    hipLaunchKernelGGL(w7_reduce2_kernel, dim3(fv_cdiv(ncol, 256)), dim3(256), 0, (hipStream_t)stream,
                       const_cast<float*>(slab), const_cast<float*>(bias_slab), t.nsplit, rpg, d->cout, dw_param, db);
    return fv_check_launch("wgrad_reduce_c7");
  }
  if (t.sub && t.v2 == 6) {
    // many splits: split sums (in place), then the phase fold
    const long rowlen = (long)t.CW * t.KW;
    const int nb1 = (int)fv_cdiv(4 * rowlen, 64), nbb1 = db ? fv_cdiv(4L * t.CW, 64) : 0;
    hipLaunchKernelGGL(subpix_split_sum_kernel, dim3(nb1 + nbb1), dim3(256), 0, (hipStream_t)stream,
                       const_cast<float*>(slab), const_cast<float*>(bias_slab), t.nsplit, rowlen, t.CW, nb1);
    if ((st = fv_check_launch("wgrad_reduce_subpix_splits"))) return st;
    const int nb2 = fv_cdiv((long)d->cout * d->cin_valid * 9, 256), nbb2 = db ? fv_cdiv(d->cout, 256) : 0;
    hipLaunchKernelGGL(subpix_fold_kernel, dim3(nb2 + nbb2), dim3(256), 0, (hipStream_t)stream, slab, bias_slab,
                       dw_param, db, t.nsplit, t.CW, t.KW, d->cout, d->cin_valid, fv_ilog2(d->cin), nb2);
    return fv_check_launch("wgrad_reduce_subpix_fold");
  }
  if (t.sub) {
    const int nb_main = fv_cdiv((long)d->cout * d->cin_valid * 9, 64);
    const int nb_bias = db ? fv_cdiv(d->cout, 64) : 0;
    hipLaunchKernelGGL(wgrad_reduce_subpix_kernel, dim3(nb_main + nb_bias), dim3(256), 0, (hipStream_t)stream, slab,
                       bias_slab, dw_param, db, t.nsplit, t.CW, t.KW, d->cout, d->cin_valid, fv_ilog2(d->cin), nb_main);
    return fv_check_launch("wgrad_reduce_subpix");
  }
  // (the packed 7x7 slab rows: k = r * 32 + s * 4 + ci, i.e. 4 "channels" x 8 "taps" per row)
  const bool pk = t.v2 == 2 && halo_wg_pk(d);
  const int K = pk ? 7 * 32 : d->ksize * d->ksize * d->cin;
  const long tot = (long)d->cout * K;
  const int nb_main = fv_cdiv(tot, 64);
  const int nb_bias = db ? fv_cdiv(d->cout, 64) : 0;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(nb_main + nb_bias), dim3(256), 0, (hipStream_t)stream, slab,
                     bias_slab, dw_param, db, t.nsplit, t.CW, t.KW, K, d->cout, d->cin_valid, pk ? 2 : fv_ilog2(d->cin),
                     d->ksize, nb_main, pk ? 8 : d->ksize);
  return fv_check_launch("wgrad_reduce");
}

}  // extern "C"

// ----------------------------------------------------------------------------------------
// ConvTranspose2dELR, kernel 4 / stride 2 / padding 1 (models_utils.py:404-516).
// out[o] = sum_j x[j] W[ci][co][o + 1 - 2j]: output phase pa (o = 2i + pa) reads the two
// low-res rows {i - 1, i} (pa = 0) or {i, i + 1} (pa = 1) -- the same 2x2 window per phase as
// the sub-pixel decomposition of nearest-x2 + 3x3 (weight_prep_subpix_kernel), with tap
// t = 3 - pa - 2 r' selected instead of folded.  So the transposed conv runs on the
// upsample-conv kernels unchanged (descriptor upsample = 1, ksize = 3, h/w = output size):
// forward = the sub-pixel phases, data gradient = the low-res stride-2 4x4 conv over dy
// (wt[ci][(tr*4 + tc)*cin_t + co] = Weff[ci][co][tr][tc]), weight gradient = the per-phase
// 2x2 slabs, mapped back to 4x4 taps here.  Weff = gain * W (* 1/max(||W[:, co]||, 1e-12)
// with norm == "demod", F.normalize over dims [0, 2, 3]: models_utils.py:461-470).
// ----------------------------------------------------------------------------------------
namespace {

// one wave per output channel: inv[co] = 1 / max(||W[:, co, :, :]||_2, 1e-12)
__global__ void convt_norm_kernel(const float* __restrict__ w, int cin, int cout, float* inv) {
  const int co = blockIdx.x, l = threadIdx.x;
  float s = 0.f;
  for (int e = l; e < cin * 16; e += 64) {
    const float v = w[((long)(e >> 4) * cout + co) * 16 + (e & 15)];
    s += v * v;
  }
  s = wave_sum(s);
  if (l == 0) inv[co] = 1.f / fmaxf(sqrtf(s), 1e-12f);
}

__device__ __forceinline__ float convt_scale(const float* inv, int co, float gain) {
  return inv ? gain * inv[co] : gain;
}

// wk [4][rows][Kpad] (k = (r'*2 + s')*cin + ci) and wt [rows_t][16*cin_t] (k = (tr*4 + tc)*cin_t + co)
__global__ void convt_weight_prep_kernel(const float* __restrict__ w, const float* __restrict__ inv, float gain,
                                         bf16* wk, int rows, int Kpad, int lgCin, bf16* wt, int rows_t,
                                         int lgCt, int cin_valid, int cout) {
  const long nk = wk ? 4L * rows * Kpad : 0;
  const long nt = wt ? (long)rows_t * (16L << lgCt) : 0;
  for (long e = blockIdx.x * (long)blockDim.x + threadIdx.x; e < nk + nt; e += (long)gridDim.x * blockDim.x) {
    float v = 0.f;
    if (e < nk) {
      const long per = (long)rows * Kpad;
      const int ph = (int)(e / per);
      const long e2 = e - ph * per;
      const int co = (int)(e2 / Kpad), k = (int)(e2 - (long)co * Kpad);
      const int tap = k >> lgCin, ci = k & ((1 << lgCin) - 1);
      if (tap < 4 && co < cout && ci < cin_valid) {
        const int tr = 3 - (ph >> 1) - 2 * (tap >> 1), tc = 3 - (ph & 1) - 2 * (tap & 1);
        v = w[((long)ci * cout + co) * 16 + tr * 4 + tc] * convt_scale(inv, co, gain);
      }
      wk[e] = (bf16)v;
    } else {
      const long e2 = e - nk;
      const int Kt = 16 << lgCt;
      const int ci = (int)(e2 / Kt), k = (int)(e2 - (long)ci * Kt);
      const int tap = k >> lgCt, co = k & ((1 << lgCt) - 1);
      if (ci < cin_valid && co < cout)
        v = w[((long)ci * cout + co) * 16 + tap] * convt_scale(inv, co, gain);
      wt[e2] = (bf16)v;
    }
  }
}

// phase slabs [4][nsplit][CW][KW] (rows co, k = ((r'*2 + s') << lgCin) + ci) -> G [ci][co][4][4]
// = dL/dWeff, one wave per 64 outputs, 4 lanes per output summing interleaved splits; + db.
__global__ void convt_wgrad_reduce_kernel(const float* __restrict__ slab, const float* __restrict__ bslab, float* dw,
                                          float* db, int nsplit, int CW, int KW, int cout, int cin_valid, int lgCin,
                                          int nb_main) {
  const int sg = threadIdx.x >> 6, l = threadIdx.x & 63;
  __shared__ float red[4][64];
  float g = 0.f;
  long dst = -1;
  if ((int)blockIdx.x < nb_main) {
    const long e = (long)blockIdx.x * 64 + l;
    if (e < (long)cin_valid * cout * 16) {
      dst = e;
      const int t = (int)(e & 15), co = (int)((e >> 4) % cout), ci = (int)((e >> 4) / cout);
      const int tr = t >> 2, tc = t & 3;
      const int ph = (1 - (tr & 1)) * 2 + (1 - (tc & 1));
      const int tap = (tr < 2) * 2 + (tc < 2);
      for (int sp = sg; sp < nsplit; sp += 4)
        g += slab[((long)(ph * nsplit + sp) * CW + co) * KW + ((tap << lgCin) + ci)];
    }
  } else {
    const int co = ((int)blockIdx.x - nb_main) * 64 + l;
    if (co < cout) {
      dst = co;
      for (int t = sg; t < 4 * nsplit; t += 4) g += bslab[(long)t * CW + co];
    }
  }
  red[sg][l] = g;
  __syncthreads();
  if (sg == 0 && dst >= 0) {
    const float v = (red[0][l] + red[1][l]) + (red[2][l] + red[3][l]);
    if ((int)blockIdx.x < nb_main) dw[dst] = v;
    else db[dst] = v;
  }
}

// in place, one wave per co: G = dL/dWeff -> dL/dW.  demod: Wn = W * inv,
// dW = gain * inv * (G - Wn <Wn, G>) (the max(norm, eps) clamp: dW = gain * inv * G); else gain * G.
__global__ void convt_weight_bwd_kernel(const float* __restrict__ w, const float* __restrict__ inv, float gain,
                                        float* g, int cin, int cout) {
  const int co = blockIdx.x, l = threadIdx.x;
  const float iv = inv ? inv[co] : 1.f;
  float dot = 0.f;
  if (inv && iv < 1e12f) {
    for (int e = l; e < cin * 16; e += 64) {
      const long a = ((long)(e >> 4) * cout + co) * 16 + (e & 15);
      dot += w[a] * iv * g[a];
    }
    dot = wave_sum(dot);
  }
  for (int e = l; e < cin * 16; e += 64) {
    const long a = ((long)(e >> 4) * cout + co) * 16 + (e & 15);
    g[a] = gain * iv * (g[a] - (inv ? w[a] * iv * dot : 0.f));
  }
}

}  // namespace

extern "C" {

int fv_convt_supported(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  if (!d->upsample || d->ksize != 3 || d->dtype != FV_BF16 || d->pro_act || d->epi_sigmoid || d->out_nchw_f32 ||
      pad_pow2_8(d->cout) != d->cout || d->ldy != d->cout)
    return 0;
  return (use_subpix(d) && use_dgrad_lowres(d) && plan_wgrad(d).sub) ? 1 : 0;
}

int fv_convt_weight_prep(const fv_conv_desc* d, const float* w, int demod, float gain, float* inv, void* wk,
                         void* wt, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fv_convt_supported(d), "conv_transpose2d k4 s2 p1: unsupported descriptor (cin=%d cout=%d %dx%d)",
             d->cin, d->cout, d->h, d->w);
  FV_REQUIRE(w && (!demod || inv), "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (demod) {
    hipLaunchKernelGGL(convt_norm_kernel, dim3(d->cout), dim3(64), 0, s, w, d->cin_valid, d->cout, inv);
    if ((st = fv_check_launch("convt_norm"))) return st;
  }
  // the halo kernels' phase layouts (conv3_halo_fwd3 MODE 1 / 2) where those kernels take the launch
  const float* cinv = demod ? inv : nullptr;
  if (wk && use_subpix_halo(d)) {
    const int nb1 = (int)std::min<long>(fv_cdiv(phase_wk_elems(d), 256), 4096);
    hipLaunchKernelGGL((weight_prep_phase_kernel<1, true>), dim3(nb1), dim3(256), 0, s, w, nullptr, (bf16*)wk,
                       4 * d->cout, 4 * (d->cin / 32), d->cout, d->cin_valid, 0, cinv, gain);
    if ((st = fv_check_launch("convt_weight_prep_phase1"))) return st;
    wk = nullptr;
  }
  if (wt && dgrad_halo_bn(d)) {
    const int nb2 = (int)std::min<long>(fv_cdiv(phase_wt_elems(d), 256), 4096);
    hipLaunchKernelGGL((weight_prep_phase_kernel<2, true>), dim3(nb2), dim3(256), 0, s, w, nullptr, (bf16*)wt, d->cin,
                       4 * (4 * d->cout / 32), d->cout, d->cin_valid, d->cout / 32, cinv, gain);
    if ((st = fv_check_launch("convt_weight_prep_phase2"))) return st;
    wt = nullptr;
  }
  if (!wk && !wt) return FV_OK;
  const int cin_t = pad_pow2_8(d->cout);
  const int rows = wrows(d->cout), Kp = kpad_of(2, d->cin);
  const int rows_t = wrows(d->cin);
  const long tot = (wk ? 4L * rows * Kp : 0) + (wt ? (long)rows_t * 16 * cin_t : 0);
  const int nb = (int)std::min<long>(fv_cdiv(tot, 256), 4096);
  hipLaunchKernelGGL(convt_weight_prep_kernel, dim3(nb), dim3(256), 0, s, w, demod ? inv : nullptr, gain, (bf16*)wk,
                     rows, Kp, fv_ilog2(d->cin), (bf16*)wt, rows_t, fv_ilog2(cin_t), d->cin_valid, d->cout);
  return fv_check_launch("convt_weight_prep");
}

int fv_convt_wgrad_reduce(const fv_conv_desc* d, const float* slab, const float* bias_slab, const float* w,
                          int demod, float gain, const float* inv, float* dw, float* db, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fv_convt_supported(d), "conv_transpose2d k4 s2 p1: unsupported descriptor");
  FV_REQUIRE(slab && w && dw && (!demod || inv) && (!db || bias_slab), "null pointer");
  const WgPlan t = plan_wgrad(d);
  hipStream_t s = (hipStream_t)stream;
  const int nb_main = fv_cdiv((long)d->cout * d->cin_valid * 16, 64);
  const int nb_bias = db ? fv_cdiv(d->cout, 64) : 0;
  hipLaunchKernelGGL(convt_wgrad_reduce_kernel, dim3(nb_main + nb_bias), dim3(256), 0, s, slab, bias_slab, dw, db,
                     t.nsplit, t.CW, t.KW, d->cout, d->cin_valid, fv_ilog2(d->cin), nb_main);
  if ((st = fv_check_launch("convt_wgrad_reduce"))) return st;
  hipLaunchKernelGGL(convt_weight_bwd_kernel, dim3(d->cout), dim3(64), 0, s, w, demod ? inv : nullptr, gain, dw,
                     d->cin_valid, d->cout);
  return fv_check_launch("convt_weight_bwd");
}

}  // extern "C"

// ========================================================================================
// fp8 (OCP e4m3) conv path: per-tensor scaled operands on v_mfma_scale_f32_16x16x128_f8f6f4
// (BASELINE config C5).  Forward and data gradient of the 3x3 convs with 128-multiple channel
// counts (ResBlock2D x 12 + Generator.in_conv: 58 % of the step's FLOPs) run on fp8 operands
// with fp32 accumulation; the weight gradient stays bf16 (its operands, the bf16 activations
// and gradients, are kept for it anyway).
//   Scaling: every fp8 tensor carries a power-of-two scale s = 2^floor(log2(448 / amax)) so
//   that |v * s| <= 448 (e4m3 max); dq = 1 / s is stored on the device and the conv epilogue
//   multiplies the fp32 accumulators by dq_x * dq_w (exact: powers of two).
// ========================================================================================
namespace {

constexpr int FP8_NPART = 1024;   // amax partials (blocks of the amax pass)

// block bid of nblk: max |x| over its grid-stride share -> part[bid]
template <typename T>
__device__ __forceinline__ void amax_body(const T* __restrict__ x, long n, float* part, int bid, int nblk) {
  float m = 0.f;
  for (long i = bid * 256L + threadIdx.x; i * 8 < n; i += (long)nblk * 256) {
    const long e = i * 8;
    if (e + 8 <= n) {
      Chunk8<T> c;
      c.load(x + e);
#pragma unroll
      for (int j = 0; j < 8; ++j) m = fmaxf(m, fabsf(c.get(j)));
    } else {
      for (long j = e; j < n; ++j) m = fmaxf(m, fabsf(Elt<T>::to_f(x[j])));
    }
  }
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0) part[bid] = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
}

template <typename T>
__global__ void __launch_bounds__(256) amax_kernel(const T* __restrict__ x, long n, float* part) {
  amax_body<T>(x, n, part, blockIdx.x, gridDim.x);
}

// every block reduces the partials itself (1024 floats from L2), block 0 publishes dq
__device__ __forceinline__ float amax_of_parts(const float* part, int np, float* sh) {
  float m = 0.f;
  for (int i = threadIdx.x; i < np; i += blockDim.x) m = fmaxf(m, part[i]);
  m = wave_max(m);
  if ((threadIdx.x & 63) == 0) sh[threadIdx.x >> 6] = m;
  __syncthreads();
  float r = 0.f;
  for (int w = 0; w < (int)(blockDim.x >> 6); ++w) r = fmaxf(r, sh[w]);
  return r;
}

template <typename T>
__global__ void __launch_bounds__(256) quantize_fp8_kernel(const T* __restrict__ x, long n, const float* part, int np,
                                                           uint8_t* __restrict__ y, float* dq) {
  __shared__ float sh[4];
  const float s = pow2_scale_of(amax_of_parts(part, np, sh));
  if (blockIdx.x == 0 && threadIdx.x == 0) dq[0] = 1.f / s;
  for (long i = blockIdx.x * 256L + threadIdx.x; i * 8 < n; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    if (e + 8 <= n) {
      Chunk8<T> c;
      c.load(x + e);
      uint2 o;
      o.x = pack4_fp8(c.get(0) * s, c.get(1) * s, c.get(2) * s, c.get(3) * s);
      o.y = pack4_fp8(c.get(4) * s, c.get(5) * s, c.get(6) * s, c.get(7) * s);
      *reinterpret_cast<uint2*>(y + e) = o;
    } else {
      for (long j = e; j < n; ++j) {
        const int v = __builtin_amdgcn_cvt_pk_fp8_f32(Elt<T>::to_f(x[j]) * s, 0.f, 0, false);
        y[j] = (uint8_t)(v & 0xff);
      }
    }
  }
}

// ---- delayed scaling (per operand site: a conv's activation or output-gradient operand) ----
// site = uint32[FP8_SITE]: [0, 16) amax history (float bits), [16] amax of the call in flight
// (float bits, atomicMax: deterministic, max is order-free), [17] history write index, [18] dq
// of the call in flight.  A call quantizes with s = pow2 scale of max(history) in ONE pass
// (values beyond 448 / s saturate, as delayed scaling does) and accumulates its own amax; the
// conv consuming the operand moves that amax into the history (fp8_site_roll, block 0 at its
// start: every quantize block has finished by then and only dq is read concurrently).  The
// site's first call quantizes exactly (amax pass + quantize pass) and fills the history.
__device__ __forceinline__ void fp8_site_roll(unsigned* st) {
  const unsigned p = st[17] % FP8_HIST;
  st[p] = st[16];
  st[16] = 0u;
  st[17] = p + 1;
}
// exact first call: fills the whole history with this call's amax
__global__ void fp8_site_seed_kernel(const float* part, int np, unsigned* st) {
  __shared__ float sh[4];
  const float m = amax_of_parts(part, np, sh);
  if (threadIdx.x < FP8_HIST) st[threadIdx.x] = __float_as_uint(m);
  if (threadIdx.x == 0) {
    st[16] = 0u;
    st[17] = 0u;
  }
}

// data-parallel global scaling (fv_fp8_set_deferred_roll): the sites' in-flight amax words,
// gathered into one float vector (all-reduced MAX across ranks by the caller), then rolled into
// every site's history at once -- identical histories, so identical scales, on every rank
__global__ void fp8_sites_inflight_kernel(int n, const unsigned long long* __restrict__ sites, float* amax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i < n) amax[i] = __uint_as_float(reinterpret_cast<const unsigned*>(sites[i])[16]);
}
__global__ void fp8_sites_roll_kernel(int n, const unsigned long long* __restrict__ sites, const float* amax) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  unsigned* st = reinterpret_cast<unsigned*>(sites[i]);
  st[16] = __float_as_uint(amax[i]);
  fp8_site_roll(st);
}
// a site's first call under global scaling: the history filled with a given (all-reduced) amax
__global__ void fp8_site_seed_from_kernel(const float* amax, unsigned* st) {
  if (threadIdx.x < FP8_HIST) st[threadIdx.x] = __float_as_uint(amax[0]);
  if (threadIdx.x == 0) {
    st[16] = 0u;
    st[17] = 0u;
  }
}
// amax of the partials -> one float
__global__ void fp8_amax_final_kernel(const float* part, int np, float* out) {
  __shared__ float sh[4];
  const float m = amax_of_parts(part, np, sh);
  if (threadIdx.x == 0) out[0] = m;
}

template <typename T>
__global__ void __launch_bounds__(256) quantize_fp8_delayed_kernel(const T* __restrict__ x, long n, unsigned* st,
                                                                   uint8_t* __restrict__ y) {
  const float s = pow2_scale_of(site_hist_max(st));
  if (blockIdx.x == 0 && threadIdx.x == 0) st[18] = __float_as_uint(1.f / s);
  float m = 0.f;
  for (long i = blockIdx.x * 256L + threadIdx.x; i * 8 < n; i += (long)gridDim.x * 256) {
    const long e = i * 8;
    if (e + 8 <= n) {
      Chunk8<T> c;
      c.load(x + e);
      float v[8];
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        v[j] = c.get(j);
        m = fmaxf(m, fabsf(v[j]));
        v[j] = fminf(fmaxf(v[j] * s, -448.f), 448.f);
      }
      uint2 o;
      o.x = pack4_fp8(v[0], v[1], v[2], v[3]);
      o.y = pack4_fp8(v[4], v[5], v[6], v[7]);
      *reinterpret_cast<uint2*>(y + e) = o;
    } else {
      for (long j = e; j < n; ++j) {
        const float f = Elt<T>::to_f(x[j]);
        m = fmaxf(m, fabsf(f));
        const int q = __builtin_amdgcn_cvt_pk_fp8_f32(fminf(fmaxf(f * s, -448.f), 448.f), 0.f, 0, false);
        y[j] = (uint8_t)(q & 0xff);
      }
    }
  }
  m = wave_max(m);
  __shared__ float red[4];
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = m;
  __syncthreads();
  if (threadIdx.x == 0)
    atomicMax(st + 16, __float_as_uint(fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]))));
}

// fp8 weights: wk [rows][9 cin] (k = tap * cin + ci) and / or the transposed, flipped wt
// [rows_t][9 cout] (k = tap' * cout + co), both scaled by s = pow2 scale of amax(|w| / sigma);
// dq[0] = 1 / s.  The amax partials of |w| come from amax_kernel<float> over w_param.
__device__ __forceinline__ void weight_prep_fp8_body(const float* __restrict__ wp, const float* sigma,
                                                     const float* part, int np, uint8_t* wk, int rows, uint8_t* wt,
                                                     int rows_t, int cout, int cin, float* dq, int bid, int nblk) {
  __shared__ float sh[4];
  const float inv = sigma ? 1.f / sigma[0] : 1.f;
  const float s = pow2_scale_of(amax_of_parts(part, np, sh) * inv);
  if (bid == 0 && threadIdx.x == 0) dq[0] = 1.f / s;
  const long nk = wk ? (long)rows * 9 * cin : 0, nt = wt ? (long)rows_t * 9 * cout : 0;
  for (long e = bid * 256L + threadIdx.x; e < nk + nt; e += (long)nblk * 256) {
    float v = 0.f;
    uint8_t* dst;
    if (e < nk) {
      const int row = (int)(e / (9 * cin)), k = (int)(e - (long)row * 9 * cin);
      const int tap = k / cin, ci = k - tap * cin;
      if (row < cout) v = wp[((long)row * cin + ci) * 9 + tap];
      dst = wk + e;
    } else {
      const long e2 = e - nk;
      const int row = (int)(e2 / (9 * cout)), k = (int)(e2 - (long)row * 9 * cout);
      const int tap = k / cout, co = k - tap * cout;
      if (row < cin) v = wp[((long)co * cin + row) * 9 + (8 - tap)];
      dst = wt + e2;
    }
    const int q = __builtin_amdgcn_cvt_pk_fp8_f32(v * inv * s, 0.f, 0, false);
    *dst = (uint8_t)(q & 0xff);
  }
}

__global__ void __launch_bounds__(256) weight_prep_fp8_kernel(const float* __restrict__ wp, const float* sigma,
                                                              const float* part, int np, uint8_t* wk, int rows,
                                                              uint8_t* wt, int rows_t, int cout, int cin, float* dq) {
  weight_prep_fp8_body(wp, sigma, part, np, wk, rows, wt, rows_t, cout, cin, dq, blockIdx.x, gridDim.x);
}

// the e4m3 weights of many convs in two launches (fv_conv_weight_prep_fp8_multi): blockIdx.y
// selects the conv, its amax partials live at ws + y * stride
struct W8Job {
  const float* w;
  const float* sigma;
  uint8_t *wk, *wt;
  float* dq;
  long nw;
  int cout, cin, nb, nb2;
};
struct W8Multi {
  int n, stride;
  W8Job j[FV_WPREP_MAX];
};
__global__ void __launch_bounds__(256) amax_multi_kernel(W8Multi m, float* ws) {
  const W8Job& j = m.j[blockIdx.y];
  if ((int)blockIdx.x >= j.nb) return;
  amax_body<float>(j.w, j.nw, ws + (long)blockIdx.y * m.stride, blockIdx.x, j.nb);
}
__global__ void __launch_bounds__(256) weight_prep_fp8_multi_kernel(W8Multi m, const float* ws) {
  const W8Job& j = m.j[blockIdx.y];
  if ((int)blockIdx.x >= j.nb2) return;
  weight_prep_fp8_body(j.w, j.sigma, ws + (long)blockIdx.y * m.stride, j.nb, j.wk, j.cout, j.wt, j.cin, j.cout, j.cin,
                       j.dq, blockIdx.x, j.nb2);
}

typedef int v8i __attribute__((ext_vector_type(8)));

__device__ __forceinline__ f32x4 mma_f8(const v8i& a, const v8i& b, f32x4 c) {
  // OCP e4m3 x e4m3 (cbsz = blgp = 0), unit block scales (e8m0 127 = 2^0)
  return __builtin_amdgcn_mfma_scale_f32_16x16x128_f8f6f4(a, b, c, 0, 0, 0, 127, 0, 127);
}

// one 16 x 16 x 128 tile, fragments in the layout the conv kernel uses: lane (r = l & 15,
// g = l >> 4) holds k {16g .. 16g+15} U {64+16g .. 64+16g+15} of A row r and of B column r.
// a [16][128], b [16][128] (b stored column-major: b[col][k]); c [16][16] row-major.
__global__ void fp8_mfma_probe_kernel(const uint8_t* a, const uint8_t* b, float* c) {
  const int l = threadIdx.x, r = l & 15, g = l >> 4;
  v8i fa, fb;
  const uint4 a0 = *reinterpret_cast<const uint4*>(a + r * 128 + 16 * g);
  const uint4 a1 = *reinterpret_cast<const uint4*>(a + r * 128 + 64 + 16 * g);
  const uint4 b0 = *reinterpret_cast<const uint4*>(b + r * 128 + 16 * g);
  const uint4 b1 = *reinterpret_cast<const uint4*>(b + r * 128 + 64 + 16 * g);
  fa = v8i{(int)a0.x, (int)a0.y, (int)a0.z, (int)a0.w, (int)a1.x, (int)a1.y, (int)a1.z, (int)a1.w};
  fb = v8i{(int)b0.x, (int)b0.y, (int)b0.z, (int)b0.w, (int)b1.x, (int)b1.y, (int)b1.z, (int)b1.w};
  f32x4 acc = mma_f8(fa, fb, f32x4{0.f, 0.f, 0.f, 0.f});
#pragma unroll
  for (int i = 0; i < 4; ++i) c[(4 * g + i) * 16 + r] = acc[i];
}

// ds_read_b64_tr_b8 probe (tests/test_fp8_gpu.py pins its lane mapping before any kernel relies
// on it): LDS byte i = i & 255 over 4 KB, lane l reads 8 transposed bytes at lane_addr[l]
typedef int v2i_t __attribute__((ext_vector_type(2)));
__global__ void tr8_probe_kernel(const int* lane_addr, int* out) {
  __shared__ __attribute__((aligned(16))) unsigned char sm[4096];
  for (int i = threadIdx.x; i < 4096; i += 64) sm[i] = (unsigned char)(i & 255);
  __syncthreads();
  const v2i_t v = __builtin_amdgcn_ds_read_tr8_b64_v2i32((FV_LDS v2i_t*)(sm + lane_addr[threadIdx.x]));
  out[2 * threadIdx.x] = v[0];
  out[2 * threadIdx.x + 1] = v[1];
}

// fp8 3x3 conv, halo-staged input (the structure of conv3_halo_fwd with a 128-channel k step):
//   k step ks = (128-channel chunk c = ks / 9, tap t = ks % 9);
//   weights stage [BN rows][128 B] (one tap x 128 ci), 16-B chunks XOR swz8(row): fragment
//   chunks g and 4 + g (the conflict-free pattern of conv_fwd_v2's 128-B rows);
//   halo of chunk c = two images (ci 0-63 / 64-127) of [(TR+2) x 66 px][64 B], h3swz chunk
//   swizzle (conflict-free fragment reads from any start), double-buffered across chunks.
// Block: BN = 128 co x BM = 256 px (4 rows x 64), 8 waves 2 (co) x 4 (px), wave 64 x 64.
// NSW: weight stages in the ring, issued NSW - 1 taps ahead (2; 3 measured slower, r4: res fwd
// / dgrad at B = 64 195 / 177 -> 199-202 / 182-185 us, fp8 step 22.36 -> 22.69 ms)
// SCH bit 1 (stagger, bit-identical): waves NW/2.. keep a tap's fragments across the next
// barrier and run its MFMAs right after it, while their SIMD partners issue the DMA and read
// their fragments; they then issue their own DMA and reads under the partners' MFMAs.
// SCH bit 0: one static s_setprio 1 for waves NW/2.. instead of the flips around each cluster.
template <int WN, int WM, int RN, int RM, int NSW = 2, int SCH = 0>
__global__ void __launch_bounds__(64 * WN * WM, 1)
conv3_halo_fp8(ConvArgs a, unsigned x_bytes) {
  constexpr int NW = WN * WM;
  constexpr int BN = WN * RN * 16, BM = WM * RM * 16, TR = BM / 64;
  constexpr int HP = (TR + 2) * 66, HQ = (HP + 15) / 16;      // pieces per 64-B halo image
  constexpr int HALO = 2 * HQ * 1024;                          // both images of one chunk
  constexpr int QH = 2 * HQ, JH = (QH + NW - 1) / NW;
  constexpr int BST = BN * 128, QB = BN / 8, JB = QB / NW;
  static_assert(QB % NW == 0, "weight pieces per wave");
  constexpr int MAIN = 2 * HALO + NSW * BST, EPI = BM * BN * 2;
  static_assert(MAIN <= 163840, "LDS");
  __shared__ __attribute__((aligned(1024))) char smem[MAIN > EPI ? MAIN : EPI];

  // the delayed-scaling site of this launch's activation operand: its dq (read below by every
  // block) was fixed by the quantize pass; block 0 moves that pass's amax into the history
  if (a.roll && blockIdx.x == 0 && threadIdx.x == 0) fp8_site_roll(a.roll);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wn = wave % WN, wm = wave / WN;
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int lid = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int tn = lid % a.ntn, tm = lid / a.ntn;
  const int tiles_w = a.W >> 6, tiles_h = a.H / TR;
  const int tw = tm % tiles_w, th = (tm / tiles_w) % tiles_h, n = tm / (tiles_w * tiles_h);
  const int co0 = tn * BN;
  const int p0 = (n * a.H + th * TR) * a.W + tw * 64;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.x), 0, (int)x_bytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(a.w), 0, 0x7fffffff, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);

  // halo pieces of this wave: piece q -> image q / HQ, 16 pixels (q % HQ) * 16 + lane / 4,
  // 16-B chunk lane % 4 (source chunk XOR h3swz)
  unsigned hoff[JH];
#pragma unroll
  for (int j = 0; j < JH; ++j) {
    const int q = wave + j * NW;
    const int img = q / HQ, hp = (q - img * HQ) * 16 + (lane >> 2), lchk = lane & 3;
    const int hr = hp / 66, hc = hp - (hp / 66) * 66;
    const int ih = th * TR + hr - 1, iw = tw * 64 + hc - 1;
    const bool ok = q < QH && hp < HP && ih >= 0 && ih < a.H && iw >= 0 && iw < a.W;
    hoff[j] = ok ? (unsigned)(((n * a.H + ih) * a.W + iw) * a.Cin + img * 64 + ((lchk ^ h3swz(hp)) << 4))
                 : 0x80000000u;
  }
  const int nh = (QH - wave + NW - 1) / NW;        // halo pieces this wave issues (JH or JH - 1)
  unsigned wbase[JB];
#pragma unroll
  for (int j = 0; j < JB; ++j) {
    const int row = (wave + j * NW) * 8 + (lane >> 3);
    wbase[j] = (unsigned)((co0 + row) * a.Kpad + (((lane & 7) ^ swz8(row)) << 4));
  }
  auto issue_b = [&](int ks) {
    const int c = ks / 9, t = ks - c * 9;
    const unsigned Bs = sbase + 2 * HALO + (ks % NSW) * BST;
    const unsigned k0 = (unsigned)(t * a.Cin + c * 128);
#pragma unroll
    for (int j = 0; j < JB; ++j) dma16s(wr, Bs + (wave + j * NW) * 1024, wbase[j], k0);
  };
  auto issue_halo = [&](int c) {
    const unsigned Hs = sbase + (c & 1) * HALO;
#pragma unroll
    for (int j = 0; j < JH; ++j)
      if (j < JH - 1 || wave + j * NW < QH) dma16s(xr, Hs + (wave + j * NW) * 1024, hoff[j], (unsigned)(c * 128));
  };

  const int lr = lane & 15, lh = lane >> 4;
  int hpb[RM];
#pragma unroll
  for (int m = 0; m < RM; ++m) {
    const int loc = wm * RM * 16 + m * 16 + lr;
    hpb[m] = (loc >> 6) * 66 + (loc & 63);
  }
  f32x4 acc[RN][RM];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int m = 0; m < RM; ++m) acc[i][m] = f32x4{0.f, 0.f, 0.f, 0.f};

  const int nch = a.Cin >> 7, nks = 9 * nch;
  const bool stag = (SCH & 2) && wave >= NW / 2;
  v8i fa[RN], fb[RM];
  auto mfma_all = [&]() {
    if constexpr (!(SCH & 1)) __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int i = 0; i < RN; ++i)
#pragma unroll
      for (int m = 0; m < RM; ++m) acc[i][m] = mma_f8(fa[i], fb[m], acc[i][m]);
    if constexpr (!(SCH & 1)) __builtin_amdgcn_s_setprio(0);
  };
  if constexpr (SCH & 1) {
    if (wave >= NW / 2) __builtin_amdgcn_s_setprio(1);
  }
  issue_b(0);
  issue_halo(0);
  if (NSW == 3 && 1 < nks) issue_b(1);
  for (int ks = 0; ks < nks; ++ks) {
    const int c = ks / 9, t = ks - c * 9;
    if constexpr (NSW == 3) {
      // stage ks (issued two steps ago) must land; stage ks + 1 (last step) may stay in flight,
      // and at t == 1 the halo of chunk c + 1 issued after it at step 9c too
      const int younger = (ks + 1 < nks ? JB : 0) + (t == 1 && c + 1 < nch ? nh : 0);
      wait_vm_dyn(younger);
    } else if (t == 1 && c + 1 < nch) {
      // step 9c+1 may leave the halo of chunk c+1 (issued last, at step 9c) in flight
      if (nh == JH) wait_vm<JH>();
      else wait_vm<(JH > 0 ? JH - 1 : 0)>();
    } else {
      wait_vm<0>();
    }
    wait_lgkm0();
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
    if constexpr ((SCH & 2) != 0) {
      if (stag && ks > 0) mfma_all();          // the previous tap's fragments
    }
    if (ks + NSW - 1 < nks) issue_b(ks + NSW - 1);
    if (t == 0 && c + 1 < nch) issue_halo(c + 1);
    const int r = t / 3, s3 = t - (t / 3) * 3;
    const char* Hs = smem + (c & 1) * HALO;
    const char* Bs = smem + 2 * HALO + (ks % NSW) * BST;
#pragma unroll
    for (int i = 0; i < RN; ++i) {
      const int row = wn * RN * 16 + i * 16 + lr;
      const uint4 u0 = *reinterpret_cast<const uint4*>(Bs + row * 128 + ((lh ^ swz8(row)) << 4));
      const uint4 u1 = *reinterpret_cast<const uint4*>(Bs + row * 128 + (((4 + lh) ^ swz8(row)) << 4));
      fa[i] = v8i{(int)u0.x, (int)u0.y, (int)u0.z, (int)u0.w, (int)u1.x, (int)u1.y, (int)u1.z, (int)u1.w};
    }
#pragma unroll
    for (int m = 0; m < RM; ++m) {
      const int hp = hpb[m] + r * 66 + s3;
      const int off = hp * 64 + ((lh ^ h3swz(hp)) << 4);
      const uint4 u0 = *reinterpret_cast<const uint4*>(Hs + off);
      const uint4 u1 = *reinterpret_cast<const uint4*>(Hs + HQ * 1024 + off);
      fb[m] = v8i{(int)u0.x, (int)u0.y, (int)u0.z, (int)u0.w, (int)u1.x, (int)u1.y, (int)u1.z, (int)u1.w};
    }
    if (!stag) mfma_all();
  }
  if (stag) mfma_all();
  if constexpr (SCH & 1) __builtin_amdgcn_s_setprio(0);
  const float dq = a.dq0[0] * a.dq1[0];
#pragma unroll
  for (int i = 0; i < RN; ++i)
#pragma unroll
    for (int m = 0; m < RM; ++m) acc[i][m] *= dq;
  __syncthreads();
  conv_epilogue<bf16, WN, WM, RN, RM, true>(a, acc, smem, co0, p0, tm, wn, wm, lane, tid);
}

// ----------------------------------------------------------------------------------------
// fp8 (e4m3) weight gradient of the 3x3 convs (BASELINE config C5): the
// sliding-row structure of conv3_halo_wgrad2 on v_mfma_scale_f32_16x16x128_f8f6f4, fed by the
// e4m3 copies of x and dy the forward / data gradient already consumed (delayed scaling, dq =
// site word 18).  A block owns 128 co x 9 taps x 64 ci and walks ROW PAIRS of one 64-column strip
// (the MFMA K = 128 pixels = output rows h and h+1):
//   D[co][(tap, ci)] += sum_{p in rows h, h+1} dy[p][co] * x[p + tap offset][ci]
// A = dy^T (rows co, k = pixel), B = x^T (rows ci, k = pixel): both transposed reads of NHWC byte
// images, ds_read_b64_tr_b8 (8 pixels x 16 channels per 16-lane group; tests/test_fp8_gpu.py
// pins the lane mapping).  A fragment (lane r = l & 15, g = l >> 4: k 16g..16g+15 U 64+16g..+15)
// = 4 such reads: pixels 16g + {0, 8} of row h, the same of row h + 1.  The 8-byte channel blocks
// of a pixel row are XOR-swizzled by the pixel (swz8d / swz8x) so the 32 lanes of a read
// (16 pixels x 2 blocks) hit 64 distinct banks; the swizzle is even, so a lane's 16-B DMA slot
// is one contiguous 16-B source chunk.  Group i = {dy rows h0+2i, h0+2i+1; x rows h0+2i+1,
// h0+2i+2} (26 pieces) travels AHEAD groups ahead; rings dy AHEAD+1 groups, x 2 AHEAD+4 rows.
// 4 waves, one per SIMD (512 registers each: the 128 x 576 tile is 288 accumulators per wave,
// which two waves per SIMD -- 256 registers each -- spill): wave (wc, wk) owns 64 co x 18 k-tiles.
// Output: the slab layout of conv3_halo_wgrad2 (fv_conv2d_wgrad_reduce), scaled by dq_x dq_dy;
// bias gradient = sum of the e4m3 dy (an all-ones B operand, ci tile 0; k-wave wk sums the co
// tiles 2 wk, 2 wk + 1 of its four).
// ----------------------------------------------------------------------------------------
struct Wg8Args {
  const uint8_t* x8;
  const uint8_t* dy8;
  const float* dqx;
  const float* dqdy;
  float* slab;
  float* bslab;
  int H, W, Cin, Cout, nseg, rows, nct, nci;
  int N, ipb;            // images, images per split (the block walks them in turn, one slab)
  unsigned xbytes, dybytes;
};

__device__ __forceinline__ int swz8x(int px) { return (((px >> 2) & 1) | (((px >> 4) & 1) << 1)) << 1; }   // 64-B rows
__device__ __forceinline__ int swz8d(int px) { return (((px >> 1) & 3) | (((px >> 4) & 1) << 2)) << 1; }   // 128-B rows
// 32-B rows (CIB = 32): a half-wave's tr_b8 pixels are two runs of 8, 16 apart, which alias mod
// 8 pixels (256 B): the block pair flips with pixel bit 4
__device__ __forceinline__ int swz8x32(int px) { return ((px >> 4) & 1) << 1; }
template <int CIB>
__device__ __forceinline__ int swz8xc(int px) {
  if constexpr (CIB == 64) return swz8x(px);
  else return swz8x32(px);
}

__device__ __forceinline__ v2i_t tr8(const char* p) {
  return __builtin_amdgcn_ds_read_tr8_b64_v2i32((FV_LDS v2i_t*)(FV_LDS char*)(p));
}

// CIB (r6): input channels per block.  64: a wave owns 64 co x 18 k-tiles =
// 288 accumulators, more than the 256 AGPRs, so the compiler rotates accumulator tiles through
// VGPRs (~860 v_accvgpr moves per 72 MFMAs).  32: the block is 128 co x 9 taps x 32 ci and a
// wave owns 64 co x 9 k-tiles = 144 accumulators (no rotation), at twice the blocks (dy rows
// read by twice as many ci tiles, through the XCD's L2) and 13 fragment reads per 9 MFMAs
// instead of 22 per 18.
template <int AHEAD, int CIB = 64>
__global__ void __launch_bounds__(256, 1)
conv3_wgrad_fp8(Wg8Args a) {
  constexpr int BC = 128, NSD = AHEAD + 1, NSX = 2 * AHEAD + 4;
  constexpr int DYR = 64 * BC, DYB = 2 * DYR;         // 8 KB per dy row, 16 KB per group
  constexpr int XQ = (66 * CIB + 1023) / 1024, XB = XQ * 1024;   // x row: 66 px x CIB B (5 / 3 pieces)
  constexpr int NPC = 16 + 2 * XQ;                    // pieces per group (26)
  __shared__ __attribute__((aligned(1024))) char smem[NSD * DYB + NSX * XB];
  char* const dyr = smem;
  char* const xr_ = smem + NSD * DYB;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wc = wave & 1, wk = wave >> 1;
  const int li = lane & 15, g = lane >> 4;
  const int strips = a.W >> 6;
  const int nblk = gridDim.x, bid = blockIdx.x;
  const int q8 = nblk / 8, r8 = nblk % 8, xcd = bid % 8;
  const int blk = (xcd < r8 ? xcd * (q8 + 1) : r8 * (q8 + 1) + (xcd - r8) * q8) + bid / 8;
  const int ntile = a.nct * a.nci;
  const int tile = blk % ntile, tc = tile % a.nct, tci = tile / a.nct;
  const int split = blk / ntile;
  const int seg = split % a.nseg, strip = (split / a.nseg) % strips, ng = split / (a.nseg * strips);
  int n = ng * a.ipb;                                 // the image being walked (issue_* read it)
  const int co0 = tc * BC, w0 = strip * 64, ci0 = tci * CIB;
  const int h0 = seg * a.rows, h1 = min(a.H, h0 + a.rows);
  const int nstep = (h1 - h0) >> 1;                   // row pairs (the host keeps segments even)
  constexpr int NWV = 4, JP = (NPC + NWV - 1) / NWV;  // 4 waves; <= 7 pieces per wave and group
  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.x8), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.dy8), 0, (int)a.dybytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds_ptr_t)smem);

  // this wave's pieces of a group: q = wave + 4 j < 26 (q < 16: dy row q >> 3, piece q & 7; else
  // x row (q - 16) / 5, piece (q - 16) % 5); source offsets relative to the row start
  const int npw = (NPC - wave + NWV - 1) / NWV;
  unsigned poff[JP];
#pragma unroll
  for (int j = 0; j < JP; ++j) {
    const int q = wave + NWV * j;
    poff[j] = 0x80000000u;
    if (q < 16) {
      const int o = (q & 7) * 1024 + lane * 16;
      const int px = o >> 7, kk = (o >> 4) & 7;
      poff[j] = (unsigned)(px * a.Cout + co0 + ((kk ^ (swz8d(px) >> 1)) << 4));
    } else if (q < NPC) {
      const int o = ((q - 16) % XQ) * 1024 + lane * 16;
      const int px = o / CIB, kk = (o >> 4) & (CIB / 16 - 1);
      const int iw = w0 - 1 + px;
      if (px < 66 && iw >= 0 && iw < a.W) poff[j] = (unsigned)(iw * a.Cin + ci0 + ((kk ^ (swz8xc<CIB>(px) >> 1)) << 4));
    }
  }
  auto xslot = [&](int y) { return (y - h0 + 1) % NSX; };
  auto issue_x = [&](int y, int j, int q) {             // x piece (q - 16) % 5 of row y
    // (the resource is rebuilt from the kernel argument here: called from inside the image
    // loop the captured one was treated as divergent and put in VGPRs)
    const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.x8), 0, (int)a.xbytes, 0x00020000);
    const bool rok = y >= 0 && y < a.H;
    dma16s(xr, sbase + NSD * DYB + xslot(y) * XB + ((q - 16) % XQ) * 1024, rok ? poff[j] : 0x80000000u,
           rok ? (unsigned)(((n * a.H + y) * a.W) * a.Cin) : 0u);
  };
  auto issue_group = [&](int i) {
    const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<uint8_t*>(a.dy8), 0, (int)a.dybytes, 0x00020000);
    const int h = h0 + 2 * i;
#pragma unroll
    for (int j = 0; j < JP; ++j) {
      const int q = wave + NWV * j;
      if (j < npw) {
        if (q < 16) {
          const int r = q >> 3;
          dma16s(dr, sbase + (i % NSD) * DYB + r * DYR + (q & 7) * 1024, poff[j],
                 (unsigned)(((n * a.H + h + r) * a.W + w0) * a.Cout));
        } else {
          issue_x(h + 1 + (q - 16) / XQ, j, q);
        }
      }
    }
  };
  // prologue of one image: x rows h0 - 1 (as row 0 of a group) and h0 (as row 1), the first
  // AHEAD groups
  auto prologue = [&]() {
#pragma unroll
    for (int j = 0; j < JP; ++j) {
      const int q = wave + NWV * j;
      if (j < npw && q >= 16) issue_x(h0 - 1 + (q - 16) / XQ, j, q);
    }
#pragma unroll
    for (int i = 0; i < AHEAD; ++i)
      if (i < nstep) issue_group(i);
  };
  prologue();

  constexpr int KTT = CIB / 16;                         // 16-ci k-tiles per tap
  constexpr int NK = 9 * KTT / 2;                       // k-tiles NK WK .. NK WK + NK - 1 of a wave
  f32x4 acc[4][NK];
#pragma unroll
  for (int q = 0; q < 4; ++q)
#pragma unroll
    for (int j = 0; j < NK; ++j) acc[q][j] = f32x4{0.f, 0.f, 0.f, 0.f};
  // bias gradient: k-wave WK sums co tiles 2 WK, 2 WK + 1 of its four (an all-ones e4m3 B operand)
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const bool do_bias = a.bslab && tci == 0;
  const int pl = 16 * g + (li >> 1);                    // this lane's pixel row of a tr_b8 block
  // r6: a split may hold ipb images (B = 64: half the fp32 slabs); each image restarts the
  // rings once every wave has passed the previous image's last step (all its DMAs waited)
  for (int im = 0; im < a.ipb; ++im) {
    if (im > 0) {
      if (ng * a.ipb + im >= a.N) break;
      n = ng * a.ipb + im;
      wait_lgkm0();
      __builtin_amdgcn_s_barrier();
      asm volatile("" ::: "memory");
      prologue();
    }
    with_const<0, 2>(wk, [&](auto wkc) {
      constexpr int WK = decltype(wkc)::value;
      for (int i = 0; i < nstep; ++i) {
        const int younger = min(AHEAD - 1, nstep - 1 - i);
        wait_vm_dyn(younger * npw);
        wait_lgkm0();
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        if (i + AHEAD < nstep) issue_group(i + AHEAD);
        const char* d0 = dyr + (i % NSD) * DYB;
        const char* d1 = d0 + DYR;
        // the fragment offsets are recomputed every step (an opaque copy of the pixel row)
        // instead of being hoisted out of the loop: 26 loop-invariant offsets would spill the
        // accumulators
        int plv = pl;
        asm volatile("" : "+v"(plv));
        v8i af[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) {
          const int cb = 2 * (wc * 4 + q) + (li & 1);   // 8-byte co block of the 128-co tile
          const int o0 = plv * BC + ((cb ^ swz8d(plv)) << 3), o1 = (plv + 8) * BC + ((cb ^ swz8d(plv + 8)) << 3);
          const v2i_t r0 = tr8(d0 + o0), r1 = tr8(d0 + o1), r2 = tr8(d1 + o0), r3 = tr8(d1 + o1);
          af[q] = v8i{r0[0], r0[1], r1[0], r1[1], r2[0], r2[1], r3[0], r3[1]};
        }
        // x fragment of k-tile j: tap (r, s), 16-ci block u; rows h - 1 + r (k < 64) and h + r
        auto xfrag = [&](int j) {
          const int kt = NK * WK + j, tap = kt / KTT, u = kt % KTT, r = tap / 3, s3 = tap - (tap / 3) * 3;
          const char* xa = xr_ + ((2 * i + r) % NSX) * XB;
          const char* xb = xr_ + ((2 * i + 1 + r) % NSX) * XB;
          const int cb = 2 * u + (li & 1);
          const int p0 = plv + s3, p1 = plv + 8 + s3;
          const int o0 = p0 * CIB + ((cb ^ swz8xc<CIB>(p0)) << 3), o1 = p1 * CIB + ((cb ^ swz8xc<CIB>(p1)) << 3);
          const v2i_t r0 = tr8(xa + o0), r1 = tr8(xa + o1), r2 = tr8(xb + o0), r3 = tr8(xb + o1);
          return v8i{r0[0], r0[1], r1[0], r1[1], r2[0], r2[1], r3[0], r3[1]};
        };
        v8i bcur = xfrag(0);
#pragma unroll
        for (int j = 0; j < NK; ++j) {
          v8i bnext = bcur;
          if (j + 1 < NK) bnext = xfrag(j + 1);
#pragma unroll
          for (int q = 0; q < 4; ++q) acc[q][j] = mma_f8(af[q], bcur, acc[q][j]);
          bcur = bnext;
        }
        if (do_bias) {
          const v8i ones = {0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838, 0x38383838};
          accb[0] = mma_f8(af[2 * WK], ones, accb[0]);
          accb[1] = mma_f8(af[2 * WK + 1], ones, accb[1]);
        }
      }
    });
  }
  with_const<0, 2>(wk, [&](auto wkc) {
    constexpr int WK = decltype(wkc)::value;
    const float dq = a.dqx[0] * a.dqdy[0], dqb = a.dqdy[0];
    const long KW = 9L * a.Cin;
    float* sl = a.slab + (long)split * a.Cout * KW;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
      const int kt = NK * WK + j, tap = kt / KTT;
      const int kcol = tap * a.Cin + ci0 + (kt % KTT) * 16 + li;
#pragma unroll
      for (int q = 0; q < 4; ++q)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj) sl[(long)(co0 + wc * 64 + q * 16 + 4 * g + jj) * KW + kcol] = acc[q][j][jj] * dq;
    }
    if (do_bias && li == 0) {
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int jj = 0; jj < 4; ++jj)
          a.bslab[(long)split * a.Cout + co0 + wc * 64 + (2 * WK + t) * 16 + 4 * g + jj] = accb[t][jj] * dqb;
    }
  });
}

// fp8 conv eligibility: 3x3, stride 1, 'same', channel counts multiples of 128 (in and out),
// W % 64 == 0, H % 4 == 0, bf16 NHWC output, operands < 2 GB
bool fp8_ok(const fv_conv_desc* d) {
  return d->ksize == 3 && !d->upsample && !d->pro_act && !d->epi_sigmoid && !d->out_nchw_f32 && d->cin % 128 == 0 &&
         d->cin_valid == d->cin && d->cout % 128 == 0 && d->ldy == d->cout && d->w % 64 == 0 && d->h % 4 == 0 &&
         (long)d->n * d->h * d->w * d->cin < (1L << 31) && (long)d->n * d->h * d->w * d->cout * 2 < (1L << 31);
}

int conv_fp8_run(const fv_conv_desc* d, int cin, int cout, const uint8_t* x8, const float* dq_x, const uint8_t* w8,
                 const float* dq_w, const float* bias, const void* res, void* y, float* stats, hipStream_t s,
                 unsigned* roll = nullptr, float* sprec = nullptr) {
  ConvArgs a{};
  // store-pass mode 1 (r6): (sum, sum of squares) of the stored, residual-added output in the
  // staged epilogue's store loop -- the records of fv_conv2d_fwd_sr, same geometry (256-pixel
  // tiles, one record per wave and tile: the bf16 res tile's count), so in fp8 mode the next
  // ResBlock's bn1 statistics need no tensor_stats pass either
  a.spm = sprec ? 1 : 0;
  a.sprec = sprec;
  a.x = x8; a.w = w8; a.bias = bias; a.res = res; a.y = y; a.stats = stats;
  a.nrec = stats ? fv_conv2d_fp8_stats_blocks(d) : 0;
  a.dq0 = dq_x; a.dq1 = dq_w;
  a.roll = roll;
  a.N = d->n; a.H = d->h; a.W = d->w; a.Hin = d->h; a.Win = d->w;
  a.P = d->n * d->h * d->w;
  a.Cin = cin; a.lgCin = fv_ilog2(cin);
  a.Cout = cout; a.ldy = cout;
  a.K = 9 * cin; a.Kpad = 9 * cin;
  a.lgtw = 6;
  a.ntn = cout / 128;
  const int nblk = a.ntn * d->n * (d->h / 4) * (d->w / 64);
  const unsigned xb = (unsigned)((long)d->n * d->h * d->w * cin);
  // (measured and not kept, r4: a 3-deep weight ring issued 3 steps ahead with the next tap's
  // fragments read under this tap's MFMAs and the barrier after them, conv3_halo_fwd2's schedule:
  // res fwd / dgrad at B = 64 188 / 172 -> 208 / 192 us: the two waves of a SIMD already hide
  // each other's fragment reads (16 KB per 16 MFMAs of 32 cycles, half the CU's 256 B/clk of
  // LDS at the fp8 peak).)
  switch (res_sched(3)) {
    case 1: hipLaunchKernelGGL((conv3_halo_fp8<2, 4, 4, 4, 2, 1>), dim3(nblk), dim3(512), 0, s, a, xb); break;
    case 2: hipLaunchKernelGGL((conv3_halo_fp8<2, 4, 4, 4, 2, 2>), dim3(nblk), dim3(512), 0, s, a, xb); break;
    case 3: hipLaunchKernelGGL((conv3_halo_fp8<2, 4, 4, 4, 2, 3>), dim3(nblk), dim3(512), 0, s, a, xb); break;
    default: hipLaunchKernelGGL((conv3_halo_fp8<2, 4, 4, 4>), dim3(nblk), dim3(512), 0, s, a, xb); break;
  }
  return fv_check_launch("conv2d_fp8");
}

}  // namespace

extern "C" {

size_t fv_fp8_ws_bytes(void) { return FP8_NPART * sizeof(float); }

int fv_quantize_fp8(int dtype_in, const void* x, long count, uint8_t* y, float* dq, void* ws, void* stream) {
  FV_REQUIRE(x && y && dq && ws && count > 0, "quantize_fp8: bad args");
  FV_REQUIRE(dtype_in == FV_BF16 || dtype_in == FV_F32, "quantize_fp8: input must be bf16 or f32");
  hipStream_t s = (hipStream_t)stream;
  const long chunks = (count + 7) / 8;
  const int nb = (int)std::min<long>(FP8_NPART, std::max<long>(1, (chunks + 255) / 256));
  if (dtype_in == FV_BF16) {
    hipLaunchKernelGGL(amax_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)x, count, (float*)ws);
    hipLaunchKernelGGL(quantize_fp8_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)x, count, (const float*)ws,
                       nb, y, dq);
  } else {
    hipLaunchKernelGGL(amax_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)x, count, (float*)ws);
    hipLaunchKernelGGL(quantize_fp8_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)x, count,
                       (const float*)ws, nb, y, dq);
  }
  return fv_check_launch("quantize_fp8");
}

size_t fv_fp8_site_bytes(void) { return FP8_SITE * sizeof(unsigned); }

int fv_fp8_set_deferred_roll(int on) {
  g_fp8_defer_roll = on ? 1 : 0;
  return FV_OK;
}

int fv_fp8_amax(int dtype_in, const void* x, long count, float* amax, void* ws, void* stream) {
  FV_REQUIRE(x && amax && ws && count > 0, "fp8_amax: bad args");
  FV_REQUIRE(dtype_in == FV_BF16 || dtype_in == FV_F32, "fp8_amax: input must be bf16 or f32");
  hipStream_t s = (hipStream_t)stream;
  const long chunks = (count + 7) / 8;
  const int nb = (int)std::min<long>(FP8_NPART, std::max<long>(1, (chunks + 255) / 256));
  if (dtype_in == FV_BF16)
    hipLaunchKernelGGL(amax_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)x, count, (float*)ws);
  else
    hipLaunchKernelGGL(amax_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)x, count, (float*)ws);
  hipLaunchKernelGGL(fp8_amax_final_kernel, dim3(1), dim3(256), 0, s, (const float*)ws, nb, amax);
  return fv_check_launch("fp8_amax");
}

int fv_fp8_site_seed(void* site, const float* amax, void* stream) {
  FV_REQUIRE(site && amax, "fp8_site_seed: bad args");
  hipLaunchKernelGGL(fp8_site_seed_from_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, amax, (unsigned*)site);
  return fv_check_launch("fp8_site_seed_from");
}

int fv_fp8_sites_inflight(int n, const uint64_t* sites, float* amax, void* stream) {
  FV_REQUIRE(n >= 0 && (n == 0 || (sites && amax)), "fp8_sites_inflight: bad args");
  if (n == 0) return FV_OK;
  hipLaunchKernelGGL(fp8_sites_inflight_kernel, dim3(fv_cdiv(n, 64)), dim3(64), 0, (hipStream_t)stream, n,
                     (const unsigned long long*)sites, amax);
  return fv_check_launch("fp8_sites_inflight");
}

int fv_fp8_sites_roll(int n, const uint64_t* sites, const float* amax, void* stream) {
  FV_REQUIRE(n >= 0 && (n == 0 || (sites && amax)), "fp8_sites_roll: bad args");
  if (n == 0) return FV_OK;
  hipLaunchKernelGGL(fp8_sites_roll_kernel, dim3(fv_cdiv(n, 64)), dim3(64), 0, (hipStream_t)stream, n,
                     (const unsigned long long*)sites, amax);
  return fv_check_launch("fp8_sites_roll");
}

int fv_quantize_fp8_site(int dtype_in, const void* x, long count, uint8_t* y, void* site, int seeded, void* ws,
                         void* stream) {
  FV_REQUIRE(x && y && site && ws && count > 0, "quantize_fp8_site: bad args");
  FV_REQUIRE(dtype_in == FV_BF16 || dtype_in == FV_F32, "quantize_fp8_site: input must be bf16 or f32");
  hipStream_t s = (hipStream_t)stream;
  unsigned* st = (unsigned*)site;
  const long chunks = (count + 7) / 8;
  const int nb = (int)std::min<long>(FP8_NPART, std::max<long>(1, (chunks + 255) / 256));
  if (!seeded) {
    // exact first call: amax pass, quantize pass (dq into the site), history filled
    int rc = fv_quantize_fp8(dtype_in, x, count, y, (float*)(st + 18), ws, stream);
    if (rc) return rc;
    hipLaunchKernelGGL(fp8_site_seed_kernel, dim3(1), dim3(256), 0, s, (const float*)ws, nb, st);
    return fv_check_launch("fp8_site_seed");
  }
  if (dtype_in == FV_BF16)
    hipLaunchKernelGGL(quantize_fp8_delayed_kernel<bf16>, dim3(nb), dim3(256), 0, s, (const bf16*)x, count, st, y);
  else
    hipLaunchKernelGGL(quantize_fp8_delayed_kernel<float>, dim3(nb), dim3(256), 0, s, (const float*)x, count, st, y);
  return fv_check_launch("quantize_fp8_delayed");
}

int fv_conv2d_fp8_supported(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK) return 0;
  return fp8_ok(d) ? 1 : 0;
}

size_t fv_conv_fp8_wk_bytes(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK || !fp8_ok(d)) return 0;
  return (size_t)d->cout * 9 * d->cin;
}

size_t fv_conv_fp8_wt_bytes(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK || !fp8_ok(d)) return 0;
  return (size_t)d->cin * 9 * d->cout;
}

int fv_conv_weight_prep_fp8(const fv_conv_desc* d, const float* w_param, const float* sigma, uint8_t* wk,
                            uint8_t* wt, float* dq, void* ws, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fp8_ok(d), "fp8 conv: unsupported descriptor (k=%d cin=%d cout=%d %dx%d)", d->ksize, d->cin, d->cout,
             d->h, d->w);
  FV_REQUIRE(w_param && (wk || wt) && dq && ws, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  const long nw = (long)d->cout * d->cin * 9;
  const int nb = (int)std::min<long>(FP8_NPART, std::max<long>(1, (nw / 8 + 255) / 256));
  hipLaunchKernelGGL(amax_kernel<float>, dim3(nb), dim3(256), 0, s, w_param, nw, (float*)ws);
  const long tot = (wk ? nw : 0) + (wt ? nw : 0);
  const int nb2 = (int)std::min<long>(2048, fv_cdiv(tot, 256));
  hipLaunchKernelGGL(weight_prep_fp8_kernel, dim3(nb2), dim3(256), 0, s, w_param, sigma, (const float*)ws, nb, wk,
                     d->cout, wt, d->cin, d->cout, d->cin, dq);
  return fv_check_launch("weight_prep_fp8");
}

int fv_conv_weight_prep_fp8_multi(int n, const fv_conv_desc* descs, const float* const* w_params,
                                  const float* const* sigmas, uint8_t* const* wks, uint8_t* const* wts,
                                  float* const* dqs, void* ws, void* stream) {
  FV_REQUIRE(n >= 1 && n <= FV_WPREP_MAX && descs && w_params && sigmas && wks && wts && dqs && ws,
             "weight_prep_fp8_multi: bad args");
  W8Multi m{};
  m.n = n;
  m.stride = FP8_NPART;
  int nb_max = 1, nb2_max = 1;
  for (int i = 0; i < n; ++i) {
    const fv_conv_desc* d = &descs[i];
    int st = check_desc(d);
    if (st) return st;
    FV_REQUIRE(fp8_ok(d), "weight_prep_fp8_multi: conv %d: unsupported descriptor", i);
    FV_REQUIRE(w_params[i] && (wks[i] || wts[i]) && dqs[i], "weight_prep_fp8_multi: null pointer (conv %d)", i);
    W8Job& j = m.j[i];
    j.w = w_params[i], j.sigma = sigmas[i], j.wk = wks[i], j.wt = wts[i], j.dq = dqs[i];
    j.nw = (long)d->cout * d->cin * 9;
    j.cout = d->cout, j.cin = d->cin;
    // the per-conv entry's grids (fv_conv_weight_prep_fp8): the same partials, the same bits
    j.nb = (int)std::min<long>(FP8_NPART, std::max<long>(1, (j.nw / 8 + 255) / 256));
    j.nb2 = (int)std::min<long>(2048, fv_cdiv((wks[i] ? j.nw : 0) + (wts[i] ? j.nw : 0), 256));
    nb_max = std::max(nb_max, j.nb);
    nb2_max = std::max(nb2_max, j.nb2);
  }
  hipStream_t s = (hipStream_t)stream;
  hipLaunchKernelGGL(amax_multi_kernel, dim3(nb_max, n), dim3(256), 0, s, m, (float*)ws);
  hipLaunchKernelGGL(weight_prep_fp8_multi_kernel, dim3(nb2_max, n), dim3(256), 0, s, m, (const float*)ws);
  return fv_check_launch("weight_prep_fp8_multi");
}

int fv_conv2d_fwd_fp8(const fv_conv_desc* d, const uint8_t* x8, const float* x_dq, const uint8_t* wk,
                      const float* w_dq, const float* bias, const void* res, void* y, float* stats, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fp8_ok(d), "fp8 conv: unsupported descriptor");
  FV_REQUIRE(x8 && x_dq && wk && w_dq && y, "null pointer");
  FV_REQUIRE(!(res && stats), "fp8 conv: residual and BN statistics in one call are not supported");
  return conv_fp8_run(d, d->cin, d->cout, x8, x_dq, wk, w_dq, bias, res, y, stats, (hipStream_t)stream);
}

int fv_conv2d_fwd_fp8_site(const fv_conv_desc* d, const uint8_t* x8, void* site, const uint8_t* wk, const float* w_dq,
                           const float* bias, const void* res, void* y, float* stats, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fp8_ok(d), "fp8 conv: unsupported descriptor");
  FV_REQUIRE(x8 && site && wk && w_dq && y, "null pointer");
  FV_REQUIRE(!(res && stats), "fp8 conv: residual and BN statistics in one call are not supported");
  unsigned* sp = (unsigned*)site;
  return conv_fp8_run(d, d->cin, d->cout, x8, (const float*)(sp + 18), wk, w_dq, bias, res, y, stats,
                      (hipStream_t)stream, g_fp8_defer_roll ? nullptr : sp);
}

int fv_conv2d_fwd_fp8_site_sr(const fv_conv_desc* d, const uint8_t* x8, void* site, const uint8_t* wk,
                              const float* w_dq, const float* bias, const void* res, void* y, const fv_store_reduce* sr,
                              void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fp8_ok(d), "fp8 conv: unsupported descriptor");
  FV_REQUIRE(x8 && site && wk && w_dq && y && sr && sr->mode == 1 && sr->records, "fwd_fp8_sr: null pointer or mode != 1");
  // the fp8 tile (128 co x 256 px, 8 waves) writes the records of the bf16 res tile (256 px,
  // 8 waves): the geometry query must describe exactly that
  int bp = 0;
  FV_REQUIRE(sr_geometry(d, &bp) == (int)((long)d->n * d->h * d->w / 256 * 8) && bp == 32,
             "fwd_fp8_sr: store-pass records unavailable for this shape");
  unsigned* sp = (unsigned*)site;
  return conv_fp8_run(d, d->cin, d->cout, x8, (const float*)(sp + 18), wk, w_dq, bias, res, y, nullptr,
                      (hipStream_t)stream, g_fp8_defer_roll ? nullptr : sp, sr->records);
}

int fv_conv2d_bwd_data_fp8_site(const fv_conv_desc* d, const uint8_t* dy8, void* site, const uint8_t* wt,
                                const float* wt_dq, void* dx, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fp8_ok(d), "fp8 conv: unsupported descriptor");
  FV_REQUIRE(dy8 && site && wt && wt_dq && dx, "null pointer");
  unsigned* sp = (unsigned*)site;
  return conv_fp8_run(d, d->cout, d->cin, dy8, (const float*)(sp + 18), wt, wt_dq, nullptr, nullptr, dx, nullptr,
                      (hipStream_t)stream, g_fp8_defer_roll ? nullptr : sp);
}

int fv_conv2d_bwd_data_fp8(const fv_conv_desc* d, const uint8_t* dy8, const float* dy_dq, const uint8_t* wt,
                           const float* wt_dq, void* dx, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fp8_ok(d), "fp8 conv: unsupported descriptor");
  FV_REQUIRE(dy8 && dy_dq && wt && wt_dq && dx, "null pointer");
  return conv_fp8_run(d, d->cout, d->cin, dy8, dy_dq, wt, wt_dq, nullptr, nullptr, dx, nullptr, (hipStream_t)stream);
}

// images per split of the fp8 weight gradient: about 512 blocks of (128 co x 32 ci) tiles x
// splits (B = 32 res: 1 image; B = 64: 2, half the slabs of the bf16 plan's one image per
// split); a divisor of N.  FV_FP8_WG_IPB=k forces k (A/B).  The slabs of fv_conv2d_bwd_weight_fp8
// are then fp8_wg_nsplit(d) (<= the bf16 plan's, so fv_conv2d_wgrad_slab_elems still sizes
// them) and fv_conv2d_wgrad_fp8_reduce sums exactly those.
static int fp8_wg_ipb(const fv_conv_desc* d) {
  const WgPlan t = plan_wgrad(d);
  const long blocks = (long)t.ntc * (d->cin / 32) * t.nsplit;
  int ipb = (int)(blocks / 512);
  if (const char* e = getenv("FV_FP8_WG_IPB")) ipb = atoi(e);
  if (ipb < 1) ipb = 1;
  if (ipb > d->n) ipb = d->n;
  while (d->n % ipb) --ipb;
  return ipb;
}
static int fp8_wg_nsplit(const fv_conv_desc* d) {
  const WgPlan t = plan_wgrad(d);
  return t.nsteps * (d->w / 64) * (d->n / fp8_wg_ipb(d));
}

int fv_conv2d_wgrad_fp8_supported(const fv_conv_desc* d) {
  static int off = -1;          // FV_FP8_WGRAD=0: the bf16 weight gradient in fp8 mode (A/B)
  if (off < 0) {
    const char* e = getenv("FV_FP8_WGRAD");
    off = (e && e[0] == '0') ? 1 : 0;
  }
  if (off || check_desc(d) != FV_OK || !fp8_ok(d) || d->cin % 64 || d->cout % 128) return 0;
  const WgPlan t = plan_wgrad(d);
  return t.v2 == 5 && t.ntk == d->cin / 64 && t.sps % 2 == 0 && d->h % t.sps == 0 ? 1 : 0;
}

// the reduce of fv_conv2d_bwd_weight_fp8's slabs: wgrad_reduce_kernel over fp8_wg_nsplit(d) splits
int fv_conv2d_wgrad_fp8_reduce(const fv_conv_desc* d, const float* slab, const float* bias_slab, float* dw_param,
                               float* db, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fv_conv2d_wgrad_fp8_supported(d), "fp8 weight gradient reduce: unsupported descriptor");
  FV_REQUIRE(slab && dw_param, "null pointer");
  FV_REQUIRE(!db || bias_slab, "db needs the bias slab");
  const WgPlan t = plan_wgrad(d);
  const int K = d->ksize * d->ksize * d->cin;
  const long tot = (long)d->cout * K;
  const int nb_main = fv_cdiv(tot, 64);
  const int nb_bias = db ? fv_cdiv(d->cout, 64) : 0;
  hipLaunchKernelGGL(wgrad_reduce_kernel, dim3(nb_main + nb_bias), dim3(256), 0, (hipStream_t)stream, slab,
                     bias_slab, dw_param, db, fp8_wg_nsplit(d), t.CW, t.KW, K, d->cout, d->cin_valid,
                     fv_ilog2(d->cin), d->ksize, nb_main, d->ksize);
  return fv_check_launch("wgrad_reduce_fp8");
}

int fv_conv2d_bwd_weight_fp8(const fv_conv_desc* d, const uint8_t* x8, const float* x_dq, const uint8_t* dy8,
                             const float* dy_dq, float* slab, float* bias_slab, void* stream) {
  int st = check_desc(d);
  if (st) return st;
  FV_REQUIRE(fv_conv2d_wgrad_fp8_supported(d), "fp8 weight gradient: unsupported descriptor");
  FV_REQUIRE(x8 && x_dq && dy8 && dy_dq && slab, "null pointer");
  const WgPlan t = plan_wgrad(d);
  const long P = (long)d->n * d->h * d->w;
  Wg8Args a{};
  a.x8 = x8; a.dy8 = dy8; a.dqx = x_dq; a.dqdy = dy_dq; a.slab = slab; a.bslab = bias_slab;
  a.H = d->h; a.W = d->w; a.Cin = d->cin; a.Cout = d->cout;
  a.nseg = t.nsteps; a.rows = t.sps; a.nct = t.ntc;
  a.xbytes = (unsigned)(P * d->cin);
  a.dybytes = (unsigned)(P * d->cout);
  a.N = d->n;
  a.ipb = fp8_wg_ipb(d);
  const int nsplit = fp8_wg_nsplit(d);
  // 32-channel input tiles (144 accumulators per wave) unless FV_FP8_WG_CIB=64 (A/B)
  const char* e = getenv("FV_FP8_WG_CIB");
  if (e && atoi(e) == 64) {
    a.nci = d->cin / 64;
    hipLaunchKernelGGL((conv3_wgrad_fp8<3, 64>), dim3(t.ntc * a.nci * nsplit), dim3(256), 0, (hipStream_t)stream, a);
  } else {
    a.nci = d->cin / 32;
    const char* ea = getenv("FV_FP8_WG_AHEAD");   // row-pair groups in flight (A/B)
    const int ahead = ea ? atoi(ea) : 2;            // (r6: res fp8 wgrad 198.8 -> 191.8 us vs 3, step -0.05 ms)
    const dim3 grid(t.ntc * a.nci * nsplit);
    if (ahead == 2) hipLaunchKernelGGL((conv3_wgrad_fp8<2, 32>), grid, dim3(256), 0, (hipStream_t)stream, a);
    else if (ahead == 4) hipLaunchKernelGGL((conv3_wgrad_fp8<4, 32>), grid, dim3(256), 0, (hipStream_t)stream, a);
    else hipLaunchKernelGGL((conv3_wgrad_fp8<3, 32>), grid, dim3(256), 0, (hipStream_t)stream, a);
  }
  return fv_check_launch("conv2d_bwd_weight_fp8");
}

// BN-statistics records of fv_conv2d_fwd_fp8: one per wave row of the 128 co x 256 px tile
// (WM = 4 rows of 64 pixels)
int fv_conv2d_fp8_stats_block_pixels(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK || !fp8_ok(d)) return 0;
  return 64;
}

int fv_conv2d_fp8_stats_blocks(const fv_conv_desc* d) {
  if (check_desc(d) != FV_OK || !fp8_ok(d)) return 0;
  return fv_cdiv((long)d->n * d->h * d->w, 64);
}

int fv_tr8_probe(const int* lane_addr, int* out, void* stream) {
  FV_REQUIRE(lane_addr && out, "tr8_probe: null pointer");
  hipLaunchKernelGGL(tr8_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, lane_addr, out);
  return fv_check_launch("tr8_probe");
}

int fv_fp8_mfma_probe(const uint8_t* a, const uint8_t* b, float* c, void* stream) {
  FV_REQUIRE(a && b && c, "null pointer");
  hipLaunchKernelGGL(fp8_mfma_probe_kernel, dim3(1), dim3(64), 0, (hipStream_t)stream, a, b, c);
  return fv_check_launch("fp8_mfma_probe");
}

}  // extern "C"
