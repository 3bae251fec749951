// 3x3x3 convolution (stride 1, padding 1) of the AFE ResBlock3D trunk for gfx950.
//
// Reference behaviour replaced: nn.Conv3d(C, C, 3, 1, 1) inside ConvBlock3D "NAC"
// (modules.py:52-56, _ResBlock 116-126, ResBlock3D 133-135) as instantiated by
// AFE.res (models.py:935, 943-944): x [N, C=32, D=16, H, W] after mid_conv's view.
//
// Layout: activations NDHWC (torch channels_last_3d), so a depth slice is an NHWC image and
// the BN / activation passes of bn.hip apply unchanged with h := D * H.
//
// Fast path (bf16, C = 32 in and out, W = 64, H % 4 == 0):
//   conv3d_c32_fwd  -- forward, and the data gradient with the transposed flipped weights.
//     GEMM D[co][voxel] = Wk[co][(tap, ci)] . X[(tap, ci)][voxel], K = 27 x 32.  A block of
//     4 waves owns (image n, 4 output rows, a depth chunk) and slides along depth: each step
//     stages ONE new input depth slice (6 rows x 64 voxels x 64 B, 24 KB) by LDS-DMA into a
//     4-slot ring while the previous three are consumed, so an input voxel is fetched about
//     1.5x (row halo) instead of 27x.  All 27 x 32 x 32 weights live in registers (54 MFMA
//     A fragments, one wave per SIMD), so the only LDS reads are the activation fragments, and
//     only those of the centre column tap: 4 ds_read_b128 per 24 v_mfma_f32_16x16x32_bf16, the
//     kw = 0 / 2 fragments made by DPP lane shifts (r2-r3 read all three: 4 per 8 MFMAs, half
//     the CU's LDS bandwidth at the MFMA peak, each read a latency the single wave per SIMD
//     must cover).  Epilogue: bias, optional residual,
//     BN (sum, sum of squares) partials per wave, bf16 store.  Used when the depth chunk has
//     no 3k - 2 length (below).
//   conv3d_c32_fwd_dr -- the same GEMM walked by INPUT slice: each slice's 12 fragments per kh
//     (4 from LDS, 8 by DPP) feed the three outputs it touches through three rotating
//     accumulator sets, so the fragment work is paid once per slice instead of three times; a
//     2-slot slice ring plus the residual rows by LDS-DMA, waits that let the previous
//     epilogue's stores pend, and a fence-free barrier (the chunk walk is peeled so the
//     accumulator rotation is static: chunk lengths 3k - 2).  r4: [32, 32, 16, 64, 64]
//     forward 143-146 -> 118-122 us (0.39 of the bf16 peak).
//   conv3d_c32_wgrad -- dW[co][tap][ci] = sum_v dy[v][co] x[v + off(tap)][ci] (+ db), K =
//     voxels.  A block of 8 waves owns 4 rows of one or more images and slides along depth
//     with a 4-slot x ring (6 rows x 80 voxel rows incl. zero halo columns) and a 2-slot dy
//     ring; both images are read with ds_read_b64_tr_b16 (voxels along k).  Wave w owns taps
//     {w, w+8, w+16, w+24}; the dy fragments of a 32-voxel k step are shared by its taps.
//     Per-block fp32 slabs [blk][32][27 x 32] are reduced deterministically (two passes).
// Generic path (any C, W, fp32 parity mode or bf16): direct VALU kernels.
#include <stdlib.h>

#include <type_traits>

#include "common.h"

namespace {

typedef __attribute__((address_space(3))) void* lds3_t;

__device__ __forceinline__ void dma16s3(__amdgpu_buffer_rsrc_t r, unsigned lds, unsigned voff) {
  asm volatile("s_mov_b32 m0, %2\n\ts_nop 0\n\tbuffer_load_dwordx4 %0, %1, 0 offen lds"
               :
               : "v"(voff), "s"(r), "s"(lds)
               : "memory", "m0");
}
__device__ __forceinline__ void vm_wait0() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

// 16-B chunk swizzle of a 64-B row (4 chunks), conflict-free ds_read_b128 from any start row
__device__ __forceinline__ int cswz(int row) { return (0x1320 >> (((row >> 2) & 3) * 4)) & 3; }

// transposed image of 64-B rows (32 bf16 columns): 32-B halves swapped on rows 8..15 mod 16
__device__ __forceinline__ int tim_off(int row, int col) {   // col % 4 == 0
  return row * 64 + ((((col >> 4) ^ ((row >> 3) & 1)) << 5) | ((col & 15) << 1));
}
// 16 columns x 32 rows (rows r0 .. r0 + 31) -> MFMA k-fragment of column cbase + (lane & 15)
__device__ __forceinline__ bf16x8 tfrag32(const char* base, int r0, int cbase, int lane) {
  const int g = lane >> 4, li = lane & 15;
  const int c = cbase + 4 * (li & 3);
  FV_LDS char* lb = (FV_LDS char*)(base);
  const s16x4 t0 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + tim_off(r0 + 8 * g + (li >> 2), c)));
  const s16x4 t1 = __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(lb + tim_off(r0 + 8 * g + 4 + (li >> 2), c)));
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
  return __builtin_bit_cast(bf16x8, v);
}

// B fragments of the kw = 0 / 2 taps from the kw = 1 (centre) fragments of the same row in
// registers: a fragment is 16 voxels (lanes li of each 16-lane row g = channel group), so the
// column shift is a DPP move within the row (row_shr:1 / row_shl:1), the voxel crossing into the
// neighbouring fragment comes from it (row_shl:15 / row_shr:15), and the out-of-row voxels -1 and
// 64 -- the zero padding -- are what bound_ctrl writes.  Bit-identical to the LDS reads.
typedef int v4i3_t __attribute__((ext_vector_type(4)));
template <int CTRL>
__device__ __forceinline__ v4i3_t dpp4x(const bf16x8& x) {
  const v4i3_t a = __builtin_bit_cast(v4i3_t, x);
  v4i3_t o;
#pragma unroll
  for (int k = 0; k < 4; ++k) o[k] = __builtin_amdgcn_update_dpp(0, a[k], CTRL, 0xf, 0xf, true);
  return o;
}
// voxel 16 j + li - 1 (kw = 0)
__device__ __forceinline__ bf16x8 shift_m1(const bf16x8& cur, const bf16x8* prev) {
  v4i3_t o = dpp4x<0x111>(cur);                       // row_shr:1
  if (prev) o |= dpp4x<0x10f>(*prev);                 // row_shl:15: lane 0 <- lane 15
  return __builtin_bit_cast(bf16x8, o);
}
// voxel 16 j + li + 1 (kw = 2)
__device__ __forceinline__ bf16x8 shift_p1(const bf16x8& cur, const bf16x8* next) {
  v4i3_t o = dpp4x<0x101>(cur);                       // row_shl:1
  if (next) o |= dpp4x<0x11f>(*next);                 // row_shr:15: lane 15 <- lane 0
  return __builtin_bit_cast(bf16x8, o);
}

// ------------------------------------------------------------------------------------------
// forward / data gradient, bf16, C = 32, W = 64
// ------------------------------------------------------------------------------------------
constexpr int C3_TH = 4;                          // output rows per block (one wave per row)
constexpr int C3_ROWB = 64 * 64;                  // one image row: 64 voxels x 32 ch bf16
constexpr int C3_SLOT = (C3_TH + 2) * C3_ROWB;    // 24 KB input depth slice (row halo)
constexpr int C3_NS = 4;                          // ring slots

struct C3Args {
  const bf16* x;
  const bf16* w;       // [27][32 out][32 in] bf16
  const float* bias;   // [32] or null
  const bf16* res;     // NDHWC like y, or null
  bf16* y;
  float* stats;        // [blocks * 4][2][32] or null
  int N, D, H;
  int dchunk, ndc;
  unsigned xbytes;
};

// NI: 16-channel output tiles per wave.  NI = 2 (used): 4 waves, one per SIMD, 358 registers,
// all 32 output channels.  (NI = 1 -- 8 waves, the two co halves of a row on two waves, two per
// SIMD, the activation fragments read by both -- measured slower, r4: forward 142-148 vs
// 158-165 us at [32, 32, 16, 64, 64].)
template <int NI>
__global__ void __launch_bounds__(64 * 4 * (2 / NI), 1) conv3d_c32_fwd(C3Args a) {
  constexpr int NWV = 4 * (2 / NI);
  __shared__ __attribute__((aligned(1024))) char smem[C3_NS * C3_SLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row = wave & 3, coh = wave >> 2;          // output row of the block, co half (NI = 1)
  const int cb0 = coh * NI * 16;                      // the wave's first output channel
  const int nht = a.H / C3_TH;
  int b = blockIdx.x;
  const int dc = b % a.ndc;
  b /= a.ndc;
  const int ht = b % nht, n = b / nht;
  const int h0 = ht * C3_TH, d0 = dc * a.dchunk, d1 = d0 + a.dchunk;
  const int li = lane & 15, g = lane >> 4;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds3_t)smem);

  // input depth di (-1 .. D) -> slot (di + 1) & 3; piece q of 1 KB = row q >> 2 (h = h0 - 1 + row),
  // voxels 16 (q & 3) + lane / 4, LDS chunk lane & 3 holding source chunk (lane & 3) ^ cswz(voxel)
  auto issue = [&](int di) {
    const unsigned lb = sbase + ((di + 1) & 3) * C3_SLOT;
#pragma unroll
    for (int j = 0; j < 24 / NWV; ++j) {
      const int q = wave + NWV * j;
      const int r = q >> 2, vv = 16 * (q & 3) + (lane >> 2);
      const int c = (lane & 3) ^ cswz(vv);
      const int h = h0 - 1 + r;
      const bool ok = di >= 0 && di < a.D && h >= 0 && h < a.H;
      const unsigned off = ok ? (unsigned)((((((n * a.D + di) * a.H + h) << 6) + vv) << 5) + c * 8) * 2u : 0x80000000u;
      dma16s3(xr, lb + q * 1024, off);
    }
  };

  // weights: A fragments wf[tap][i] (rows co = 16 i + li, k = ci 8 g .. 8 g + 7)
  bf16x8 wf[27][NI];
#pragma unroll
  for (int t = 0; t < 27; ++t)
#pragma unroll
    for (int i = 0; i < NI; ++i)
      wf[t][i] = *reinterpret_cast<const bf16x8*>(a.w + ((t * 32 + cb0 + 16 * i + li) * 32 + 8 * g));
  float bv[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) bv[i][k] = a.bias ? a.bias[cb0 + 16 * i + 4 * g + k] : 0.f;
  float ss[NI][4], sq[NI][4];
#pragma unroll
  for (int i = 0; i < NI; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) ss[i][k] = sq[i][k] = 0.f;

  issue(d0 - 1);
  issue(d0);
  issue(d0 + 1);
  for (int d = d0; d < d1; ++d) {
    vm_wait0();
    __syncthreads();
    if (d + 2 <= d1) issue(d + 2);
    f32x4 acc[NI][4];
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int kd = 0; kd < 3; ++kd) {
      const char* sb = smem + ((d + kd) & 3) * C3_SLOT;
#pragma unroll
      for (int kh = 0; kh < 3; ++kh) {
        const char* rb = sb + (row + kh) * C3_ROWB;
        // the row's centre fragments (kw = 1) from LDS; kw = 0 / 2 by lane shifts (shift_m1 / p1)
        bf16x8 cx[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          const int v = 16 * j + li;
          cx[j] = *reinterpret_cast<const bf16x8*>(rb + v * 64 + ((g ^ cswz(v)) << 4));
        }
#pragma unroll
        for (int kw = 0; kw < 3; ++kw) {
          const int t = kd * 9 + kh * 3 + kw;
          bf16x8 bx[4];
#pragma unroll
          for (int j = 0; j < 4; ++j)
            bx[j] = kw == 1 ? cx[j] : kw == 0 ? shift_m1(cx[j], j > 0 ? &cx[j - 1] : nullptr)
                                              : shift_p1(cx[j], j < 3 ? &cx[j + 1] : nullptr);
#pragma unroll
          for (int i = 0; i < NI; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j)
              acc[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][i], bx[j], acc[i][j], 0, 0, 0);
        }
      }
    }
    // epilogue: lane holds co = cb0 + 16 i + 4 g + k of voxel 16 j + li in row h0 + row
    const long rowv = ((long)(n * a.D + d) * a.H + h0 + row) << 6;
#pragma unroll
    for (int i = 0; i < NI; ++i) {
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long e = ((rowv + 16 * j + li) << 5) + cb0 + 16 * i + 4 * g;
        float o[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) o[k] = acc[i][j][k] + bv[i][k];
        if (a.res) {
          const uint2 rv = *reinterpret_cast<const uint2*>(a.res + e);
          o[0] += __uint_as_float(rv.x << 16);
          o[1] += __uint_as_float(rv.x & 0xffff0000u);
          o[2] += __uint_as_float(rv.y << 16);
          o[3] += __uint_as_float(rv.y & 0xffff0000u);
        }
        bf16 t4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          t4[k] = (bf16)o[k];
          const float r = (float)t4[k];
          ss[i][k] += r;
          sq[i][k] += r * r;
        }
        *reinterpret_cast<uint2*>(a.y + e) = *reinterpret_cast<const uint2*>(t4);
      }
    }
  }
  if (a.stats) {
    const long rec = (long)blockIdx.x * C3_TH + row;
#pragma unroll
    for (int i = 0; i < NI; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float S = row16_sum(ss[i][k]), Q = row16_sum(sq[i][k]);
        if (li == 0) {
          a.stats[(rec * 2) * 32 + cb0 + 16 * i + 4 * g + k] = S;
          a.stats[(rec * 2 + 1) * 32 + cb0 + 16 * i + 4 * g + k] = Q;
        }
      }
  }
}

// Depth-reuse variant: the wave walks INPUT depth slices and applies each slice's 12 activation
// fragments (4 centre + 8 DPP-shifted, per kh) to the three outputs it feeds -- s + 1 (kd = 0),
// s (kd = 1), s - 1 (kd = 2) -- with three rotating accumulator sets, so the DPP shifts and LDS
// reads are paid once per slice instead of once per (slice, kd): 1/3 of the VALU per MFMA of
// conv3d_c32_fwd (whose DPP issue, 8 cycles per 16x16x32 MFMA free beside it, was the limiter).
// Only the current slice is read, so a 2-slot ring (48 KB).  Output s - 1 is complete after
// slice s and leaves through the same epilogue.
constexpr int C3R_NS = 2;
template <bool fN, bool fM, bool fP>
__device__ __forceinline__ void c3r_slice(const char* sb, int row, int lane, const bf16x8 (&wf)[27][2],
                                          f32x4 (&aN)[2][4], f32x4 (&aM)[2][4], f32x4 (&aP)[2][4]) {
  const int li = lane & 15, g = lane >> 4;
#pragma unroll
  for (int kh = 0; kh < 3; ++kh) {
    const char* rb = sb + (row + kh) * C3_ROWB;
    bf16x8 cx[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int v = 16 * j + li;
      cx[j] = *reinterpret_cast<const bf16x8*>(rb + v * 64 + ((g ^ cswz(v)) << 4));
    }
#pragma unroll
    for (int kw = 0; kw < 3; ++kw) {
      bf16x8 bx[4];
#pragma unroll
      for (int j = 0; j < 4; ++j)
        bx[j] = kw == 1 ? cx[j] : kw == 0 ? shift_m1(cx[j], j > 0 ? &cx[j - 1] : nullptr)
                                          : shift_p1(cx[j], j < 3 ? &cx[j + 1] : nullptr);
      const int t = kh * 3 + kw;
      if (fP) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j) aP[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[t][i], bx[j], aP[i][j], 0, 0, 0);
      }
      if (fM) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            aM[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[9 + t][i], bx[j], aM[i][j], 0, 0, 0);
      }
      if (fN) {
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
          for (int j = 0; j < 4; ++j)
            aN[i][j] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[18 + t][i], bx[j], aN[i][j], 0, 0, 0);
      }
    }
  }
}

template <int K>
__device__ __forceinline__ void vm_wait() { asm volatile("s_waitcnt vmcnt(%0)" ::"n"(K) : "memory"); }

constexpr int C3R_RES = C3_TH * C3_ROWB;   // residual rows of one output slice (16 KB)
template <bool STATS, bool RES>
__global__ void __launch_bounds__(256, 1) conv3d_c32_fwd_dr(C3Args a) {
  // [2 input slices][2 residual slices][bias]
  __shared__ __attribute__((aligned(1024))) char smem[C3R_NS * C3_SLOT + 2 * C3R_RES + 128];
  float* const sbias = reinterpret_cast<float*>(smem + C3R_NS * C3_SLOT + 2 * C3R_RES);
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int row = wave;
  const int nht = a.H / C3_TH;
  int b = blockIdx.x;
  const int dc = b % a.ndc;
  b /= a.ndc;
  const int ht = b % nht, n = b / nht;
  const int h0 = ht * C3_TH, d0 = dc * a.dchunk, d1 = d0 + a.dchunk;
  const int li = lane & 15, g = lane >> 4;

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t rr =
      __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.res ? a.res : a.x), 0, (int)a.xbytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds3_t)smem);
  // input depth di (-1 .. D) -> slot (di + 1) & 1; pieces as conv3d_c32_fwd
  auto issue = [&](int di) {
    const unsigned lb = sbase + ((di + 1) & 1) * C3_SLOT;
#pragma unroll
    for (int j = 0; j < 6; ++j) {
      const int q = wave + 4 * j;
      const int r = q >> 2, vv = 16 * (q & 3) + (lane >> 2);
      const int c = (lane & 3) ^ cswz(vv);
      const int h = h0 - 1 + r;
      const bool ok = di >= 0 && di < a.D && h >= 0 && h < a.H;
      const unsigned off = ok ? (unsigned)((((((n * a.D + di) * a.H + h) << 6) + vv) << 5) + c * 8) * 2u : 0x80000000u;
      dma16s3(xr, lb + q * 1024, off);
    }
  };
  // the wave's residual row of output d -> residual slot d & 1 (4 pieces, plain [voxel][64 B])
  auto issue_res = [&](int d) {
    const unsigned lb = sbase + C3R_NS * C3_SLOT + (d & 1) * C3R_RES + row * C3_ROWB;
#pragma unroll
    for (int p = 0; p < 4; ++p) {
      const int vv = 16 * p + (lane >> 2);
      const unsigned off = (unsigned)((((((n * a.D + d) * a.H + h0 + row) << 6) + vv) << 5) + (lane & 3) * 8) * 2u;
      dma16s3(rr, lb + p * 1024, off);
    }
  };

  bf16x8 wf[27][2];
#pragma unroll
  for (int t = 0; t < 27; ++t)
#pragma unroll
    for (int i = 0; i < 2; ++i)
      wf[t][i] = *reinterpret_cast<const bf16x8*>(a.w + ((t * 32 + 16 * i + li) * 32 + 8 * g));
  if (tid < 32) sbias[tid] = a.bias ? a.bias[tid] : 0.f;
  float ss[2][4], sq[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int k = 0; k < 4; ++k) ss[i][k] = sq[i][k] = 0.f;

  // output d: bias, residual (from LDS), bf16 store (8 global stores per lane, the only vector
  // memory operations besides the DMA in the walk: step waits count them), BN partials; the set
  // is zeroed for reuse
  auto epilogue = [&](f32x4 (&acc)[2][4], int d) {
    const long rowv = ((long)(n * a.D + d) * a.H + h0 + row) << 6;
    const char* rb = smem + C3R_NS * C3_SLOT + (d & 1) * C3R_RES + row * C3_ROWB;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const float4 bv = *reinterpret_cast<const float4*>(sbias + 16 * i + 4 * g);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long e = ((rowv + 16 * j + li) << 5) + 16 * i + 4 * g;
        float o[4] = {acc[i][j][0] + bv.x, acc[i][j][1] + bv.y, acc[i][j][2] + bv.z, acc[i][j][3] + bv.w};
        if constexpr (RES) {
          const uint2 rv = *reinterpret_cast<const uint2*>(rb + (16 * j + li) * 64 + (16 * i + 4 * g) * 2);
          o[0] += __uint_as_float(rv.x << 16);
          o[1] += __uint_as_float(rv.x & 0xffff0000u);
          o[2] += __uint_as_float(rv.y << 16);
          o[3] += __uint_as_float(rv.y & 0xffff0000u);
        }
        bf16 t4[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
          t4[k] = (bf16)o[k];
          const float r = (float)t4[k];
          if constexpr (STATS) {
            ss[i][k] += r;
            sq[i][k] += r * r;
          }
        }
        *reinterpret_cast<uint2*>(a.y + e) = *reinterpret_cast<const uint2*>(t4);
        acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
      }
    }
  };

  f32x4 A[2][4], B[2][4], C[2][4];
#pragma unroll
  for (int i = 0; i < 2; ++i)
#pragma unroll
    for (int j = 0; j < 4; ++j) A[i][j] = B[i][j] = C[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

  // one input slice s: N = output s - 1 (kd = 2), M = output s (kd = 1), P = output s + 1 (kd = 0);
  // F bits: 4 N (epilogue), 2 M, 1 P, 8 the previous step ran an epilogue (its 8 stores are
  // the operations issued after this slice's DMA, so the wait lets them pend).  The flags are
  // compile-time (the walk's first and last three slices are peeled), so the rotating
  // accumulator sets never meet at a run-time merge.  Slices outside the volume are zero-filled
  // by the DMA, so their MFMAs add nothing.  The barrier carries no memory fence: the only
  // cross-wave data is DMA-written LDS, covered by each wave's own vmcnt wait.
  auto step = [&](auto fl, int s, f32x4 (&aN)[2][4], f32x4 (&aM)[2][4], f32x4 (&aP)[2][4]) {
    constexpr int F = decltype(fl)::value;
    if constexpr ((F & 8) != 0) vm_wait<8>();
    else vm_wait<0>();
    __builtin_amdgcn_s_barrier();
    if (s + 1 <= d1) issue(s + 1);
    if (RES && s >= d0 && s < d1) issue_res(s);
    const char* sb = smem + ((s + 1) & 1) * C3_SLOT;
    c3r_slice<(F & 4) != 0, (F & 2) != 0, (F & 1) != 0>(sb, row, lane, wf, aN, aM, aP);
    if constexpr ((F & 4) != 0) epilogue(aN, s - 1);
  };
  using f001 = std::integral_constant<int, 1>;
  using f011 = std::integral_constant<int, 3>;
  using f111 = std::integral_constant<int, 7>;
  using f111e = std::integral_constant<int, 15>;
  using f110e = std::integral_constant<int, 14>;
  using f100e = std::integral_constant<int, 12>;
  // dchunk + 2 slices, a multiple of 3 and >= 6 (host)
  issue(d0 - 1);
  __syncthreads();   // sbias
  step(f001{}, d0 - 1, A, B, C);
  step(f011{}, d0, B, C, A);
  step(f111{}, d0 + 1, C, A, B);
  for (int s = d0 + 2; s < d1 - 2; s += 3) {
    step(f111e{}, s, A, B, C);
    step(f111e{}, s + 1, B, C, A);
    step(f111e{}, s + 2, C, A, B);
  }
  step(f111e{}, d1 - 2, A, B, C);
  step(f110e{}, d1 - 1, B, C, A);
  step(f100e{}, d1, C, A, B);
  if (STATS) {
    const long rec = (long)blockIdx.x * C3_TH + row;
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const float S = row16_sum(ss[i][k]), Q = row16_sum(sq[i][k]);
        if (li == 0) {
          a.stats[(rec * 2) * 32 + 16 * i + 4 * g + k] = S;
          a.stats[(rec * 2 + 1) * 32 + 16 * i + 4 * g + k] = Q;
        }
      }
  }
}

// ------------------------------------------------------------------------------------------
// weight gradient, bf16, C = 32, W = 64
// ------------------------------------------------------------------------------------------
constexpr int W3_TH = 4;
constexpr int W3_XROW = 80;                          // voxel rows per image row: w = -1 .. 78
constexpr int W3_XSLOT = (W3_TH + 2) * W3_XROW * 64;  // 30 KB
constexpr int W3_DSLOT = W3_TH * 64 * 64;             // 16 KB
constexpr int W3_NX = 4, W3_ND = 2;

struct C3WArgs {
  const bf16* x;
  const bf16* dy;
  float* slab;    // [nblk][32][864]
  float* bslab;   // [nblk][32]
  int N, D, H;
  int nper;       // images per block
  int ndc;        // depth chunks (blocks per (images, row tile)): fills the CUs at small batch
  unsigned xbytes, dybytes;
};

__global__ void __launch_bounds__(512, 1) conv3d_c32_wgrad(C3WArgs a) {
  __shared__ __attribute__((aligned(1024))) char smem[W3_NX * W3_XSLOT + W3_ND * W3_DSLOT];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int nht = a.H / W3_TH;
  const int dc = blockIdx.x % a.ndc, rest = blockIdx.x / a.ndc;
  const int ht = rest % nht, nb = rest / nht;
  const int h0 = ht * W3_TH;
  const int n0 = nb * a.nper, n1 = min(a.N, n0 + a.nper);
  const int dch = (a.D + a.ndc - 1) / a.ndc, d0 = min(a.D, dc * dch), d1 = min(a.D, d0 + dch);

  const __amdgpu_buffer_rsrc_t xr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.x), 0, (int)a.xbytes, 0x00020000);
  const __amdgpu_buffer_rsrc_t dr = __builtin_amdgcn_make_buffer_rsrc(const_cast<bf16*>(a.dy), 0, (int)a.dybytes, 0x00020000);
  const unsigned sbase = __builtin_amdgcn_readfirstlane((unsigned)(size_t)(lds3_t)smem);
  const unsigned dbase = sbase + W3_NX * W3_XSLOT;

  // x slice di of image n -> slot (di + 1) & 3: 30 pieces, row R = 16 q + lane / 4 of the
  // transposed image (r = R / 80, w = R % 80 - 1), 16-B chunk lane & 3
  auto issue_x = [&](int n, int di) {
    const unsigned lb = sbase + ((di + 1) & 3) * W3_XSLOT;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int q = wave + 8 * j;
      if (q < 30) {
        const int R = 16 * q + (lane >> 2), cp = lane & 3;
        const int c = ((((cp >> 1) ^ ((R >> 3) & 1))) << 1) | (cp & 1);
        const int r = R / W3_XROW, w = R - r * W3_XROW - 1;
        const int h = h0 - 1 + r;
        const bool ok = di >= 0 && di < a.D && h >= 0 && h < a.H && (unsigned)w < 64u;
        const unsigned off = ok ? (unsigned)((((((n * a.D + di) * a.H + h) << 6) + w) << 5) + c * 8) * 2u : 0x80000000u;
        dma16s3(xr, lb + q * 1024, off);
      }
    }
  };
  // dy slice d -> slot d & 1: 16 pieces, row R = voxel (rr * 64 + w)
  auto issue_dy = [&](int n, int d) {
    const unsigned lb = dbase + (d & 1) * W3_DSLOT;
#pragma unroll
    for (int j = 0; j < 2; ++j) {
      const int q = wave + 8 * j;
      const int R = 16 * q + (lane >> 2), cp = lane & 3;
      const int c = ((((cp >> 1) ^ ((R >> 3) & 1))) << 1) | (cp & 1);
      const int rr = R >> 6, w = R & 63;
      const unsigned off = (unsigned)((((((n * a.D + d) * a.H + h0 + rr) << 6) + w) << 5) + c * 8) * 2u;
      dma16s3(dr, lb + q * 1024, off);
    }
  };

  // taps of this wave: t = wave + 8 m (m < 4, the 4th only for waves 0..2)
  const int ntap = wave < 3 ? 4 : 3;
  f32x4 acc[4][2][2];
#pragma unroll
  for (int m = 0; m < 4; ++m)
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int c = 0; c < 2; ++c) acc[m][i][c] = f32x4{0.f, 0.f, 0.f, 0.f};
  f32x4 accb[2] = {f32x4{0.f, 0.f, 0.f, 0.f}, f32x4{0.f, 0.f, 0.f, 0.f}};
  const bool do_bias = a.bslab && wave == 7;
  bf16x8 ones;
#pragma unroll
  for (int i = 0; i < 8; ++i) ones[i] = (bf16)1.0f;
  int tkd[4], tkh[4], tkw[4];
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    const int t = wave + 8 * m;
    tkd[m] = t / 9;
    tkh[m] = (t / 3) % 3;
    tkw[m] = t % 3;
  }

  // Transposed-read addresses, hoisted: a fragment's rows start at a multiple of 16 plus the
  // tap's kw (x image rows are 80 voxels, a multiple of 16), so the half-swap swizzle of
  // tim_off is fixed per (lane, tap, column half, 4-row half) -- those lane constants are made
  // once, the slot base joins them once per depth step, and the k step's row offset is an
  // immediate (the k loop is unrolled).  The same reads as tfrag32: bit-identical.
  const int li0 = lane & 15, g0 = lane >> 4;
  auto lconst = [&](int rowl, int col) {
    return rowl * 64 + ((((col >> 4) ^ ((rowl >> 3) & 1)) << 5) | ((col & 15) << 1));
  };
  unsigned lcx[4][2][2], lcd[2][2];
#pragma unroll
  for (int h = 0; h < 2; ++h) {
    const int rl = 8 * g0 + (li0 >> 2) + 4 * h;
#pragma unroll
    for (int c = 0; c < 2; ++c) {
      const int col = 16 * c + 4 * (li0 & 3);
      lcd[c][h] = (unsigned)lconst(rl, col);
#pragma unroll
      for (int m = 0; m < 4; ++m) lcx[m][c][h] = (unsigned)(lconst(tkw[m] + rl, col) + tkh[m] * W3_XROW * 64);
    }
  }
  auto trd = [](unsigned addr) {
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16((FV_LDS s16x4*)(size_t)addr);
  };
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  auto frag = [&](unsigned a0, unsigned a1) {
    const s16x4 t0 = trd(a0), t1 = trd(a1);
    const s16x8 v = {t0[0], t0[1], t0[2], t0[3], t1[0], t1[1], t1[2], t1[3]};
    return __builtin_bit_cast(bf16x8, v);
  };

  for (int n = n0; n < n1 && d0 < d1; ++n) {
    issue_x(n, d0 - 1);
    issue_x(n, d0);
    issue_x(n, d0 + 1);
    issue_dy(n, d0);
    for (int d = d0; d < d1; ++d) {
      vm_wait0();
      __syncthreads();
      if (d + 2 <= d1) issue_x(n, d + 2);
      if (d + 1 < d1) issue_dy(n, d + 1);
      unsigned xa[4][2][2], da[2][2];
      const unsigned dslot = dbase + (d & 1) * W3_DSLOT;
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int h = 0; h < 2; ++h) {
          da[c][h] = dslot + lcd[c][h];
#pragma unroll
          for (int m = 0; m < 4; ++m) xa[m][c][h] = sbase + ((d + tkd[m]) & 3) * W3_XSLOT + lcx[m][c][h];
        }
#pragma unroll
      for (int ks = 0; ks < W3_TH * 2; ++ks) {      // 32-voxel k steps: row rr, half sg
        const int rr = ks >> 1, sg = ks & 1;
        const unsigned od = (unsigned)((rr * 64 + 32 * sg) * 64), ox = (unsigned)((rr * W3_XROW + 32 * sg) * 64);
        bf16x8 af[2];
#pragma unroll
        for (int i = 0; i < 2; ++i) af[i] = frag(da[i][0] + od, da[i][1] + od);
        if (do_bias) {
#pragma unroll
          for (int i = 0; i < 2; ++i) accb[i] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], ones, accb[i], 0, 0, 0);
        }
#pragma unroll
        for (int m = 0; m < 4; ++m) {
          if (m < 3 || ntap == 4) {
            bf16x8 bx[2];
#pragma unroll
            for (int c = 0; c < 2; ++c) bx[c] = frag(xa[m][c][0] + ox, xa[m][c][1] + ox);
#pragma unroll
            for (int i = 0; i < 2; ++i)
#pragma unroll
              for (int c = 0; c < 2; ++c)
                acc[m][i][c] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[i], bx[c], acc[m][i][c], 0, 0, 0);
          }
        }
      }
    }
    __syncthreads();   // every wave done with the rings before the next image's prologue
  }

  // D[co][ci]: lane holds co = 16 i + 4 (lane >> 4) + k, ci = 16 c + (lane & 15)
  const int li = lane & 15, g = lane >> 4;
  float* slab = a.slab + (long)blockIdx.x * 32 * 864;
#pragma unroll
  for (int m = 0; m < 4; ++m) {
    if (m < 3 || ntap == 4) {
      const int t = wave + 8 * m;
#pragma unroll
      for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int c = 0; c < 2; ++c)
#pragma unroll
          for (int k = 0; k < 4; ++k) slab[(16 * i + 4 * g + k) * 864 + t * 32 + 16 * c + li] = acc[m][i][c][k];
    }
  }
  if (do_bias && li == 0) {
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
      for (int k = 0; k < 4; ++k) a.bslab[(long)blockIdx.x * 32 + 16 * i + 4 * g + k] = accb[i][k];
  }
}

// slabs [nblk][32][864] -> partial sums [ns][32 * 864 + 32] (pass 1), -> dw / db (pass 2)
__global__ void __launch_bounds__(256) c3w_reduce1(const float* __restrict__ slab, const float* __restrict__ bslab,
                                                   int nblk, int ns, float* part) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int s = blockIdx.y;
  const int per = (nblk + ns - 1) / ns, b0 = s * per, b1 = min(nblk, b0 + per);
  const int E = 32 * 864;
  if (e < E) {
    float acc = 0.f;
    for (int b = b0; b < b1; ++b) acc += slab[(long)b * E + e];
    part[(long)s * (E + 32) + e] = acc;
  } else if (e < E + 32 && bslab) {
    float acc = 0.f;
    for (int b = b0; b < b1; ++b) acc += bslab[(long)b * 32 + (e - E)];
    part[(long)s * (E + 32) + e] = acc;
  }
}
// dw[co][ci][tap] (= reference [co][ci][kd][kh][kw]) from k = tap * 32 + ci
__global__ void __launch_bounds__(256) c3w_reduce2(const float* __restrict__ part, int ns, float* dw, float* db) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  const int E = 32 * 864;
  if (e < E) {
    float acc = 0.f;
    for (int s = 0; s < ns; ++s) acc += part[(long)s * (E + 32) + e];
    const int co = e / 864, k = e - co * 864, t = k >> 5, ci = k & 31;
    dw[(co * 32 + ci) * 27 + t] = acc;
  } else if (e < E + 32 && db) {
    float acc = 0.f;
    for (int s = 0; s < ns; ++s) acc += part[(long)s * (E + 32) + e];
    db[e - E] = acc;
  }
}

// ------------------------------------------------------------------------------------------
// generic direct kernels (fp32 parity mode, or shapes off the fast path)
// ------------------------------------------------------------------------------------------
// y[v][o] = sum_{t, i} w[t][i][o] x[v + off(t)][i] (+ bias[o]) (+ res[v][o]); 8 outputs/thread
template <typename T>
__global__ void __launch_bounds__(256) conv3d_direct_fwd(const T* __restrict__ x, const float* __restrict__ w,
                                                         const float* bias, const T* res, T* y, int N, int D,
                                                         int H, int W, int Ci, int Co) {
  const int og = Co / 8;
  const long idx = (long)blockIdx.x * 256 + threadIdx.x;
  const long V = (long)N * D * H * W;
  if (idx >= V * og) return;
  const int o0 = (int)(idx % og) * 8;
  const long v = idx / og;
  const int xw = (int)(v % W), xh = (int)((v / W) % H), xd = (int)((v / ((long)W * H)) % D);
  const long n = v / ((long)W * H * D);
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = bias ? bias[o0 + j] : 0.f;
  for (int t = 0; t < 27; ++t) {
    const int dd = xd + t / 9 - 1, hh = xh + (t / 3) % 3 - 1, ww = xw + t % 3 - 1;
    if (dd < 0 || dd >= D || hh < 0 || hh >= H || ww < 0 || ww >= W) continue;
    const T* xp = x + ((((n * D + dd) * H + hh) * W + ww) * Ci);
    const float* wp = w + (long)t * Ci * Co + o0;
    for (int i = 0; i < Ci; ++i) {
      const float xv = Elt<T>::to_f(xp[i]);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] = fmaf(xv, wp[(long)i * Co + j], acc[j]);
    }
  }
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    float o = acc[j];
    if (res) o += Elt<T>::to_f(res[v * Co + o0 + j]);
    y[v * Co + o0 + j] = Elt<T>::from_f(o);
  }
}

// block per (tap, output channel o): dw[o][i][t] = sum_v dy[v][o] x[v + off(t)][i] for all i
// (Ci <= 64); blocks of tap 0 also write db[o] = sum_v dy[v][o].  Deterministic tree sums.
template <typename T>
__global__ void __launch_bounds__(256) conv3d_direct_wgrad(const T* __restrict__ x, const T* __restrict__ dy,
                                                           float* dw, float* db, int N, int D, int H, int W,
                                                           int Ci, int Co) {
  const int t = blockIdx.x % 27, o = blockIdx.x / 27;
  const int od = t / 9 - 1, oh = (t / 3) % 3 - 1, ow = t % 3 - 1;
  const long V = (long)N * D * H * W;
  float acc[65];
  for (int i = 0; i <= Ci; ++i) acc[i] = 0.f;
  for (long v = threadIdx.x; v < V; v += 256) {
    const float g = Elt<T>::to_f(dy[v * Co + o]);
    acc[Ci] += g;
    const int xw = (int)(v % W), xh = (int)((v / W) % H), xd = (int)((v / ((long)W * H)) % D);
    const long n = v / ((long)W * H * D);
    const int dd = xd + od, hh = xh + oh, ww = xw + ow;
    if (dd < 0 || dd >= D || hh < 0 || hh >= H || ww < 0 || ww >= W) continue;
    const T* xp = x + ((((n * D + dd) * H + hh) * W + ww) * Ci);
    for (int i = 0; i < Ci; ++i) acc[i] = fmaf(g, Elt<T>::to_f(xp[i]), acc[i]);
  }
  __shared__ float red[256];
  for (int i = 0; i <= Ci; ++i) {
    red[threadIdx.x] = acc[i];
    __syncthreads();
    for (int s = 128; s > 0; s >>= 1) {
      if (threadIdx.x < s) red[threadIdx.x] += red[threadIdx.x + s];
      __syncthreads();
    }
    if (threadIdx.x == 0) {
      if (i < Ci) dw[((long)o * Ci + i) * 27 + t] = red[0];
      else if (t == 0 && db) db[o] = red[0];
    }
    __syncthreads();
  }
}

// w [co][ci][27] fp32 -> out, element (t', o, i): flip = 0: o = co, i = ci, t' = t;
// flip = 1 (data gradient): o = ci, i = co, t' = 26 - t.  out_major: [t'][o][i], else [t'][i][o]
template <typename T>
__global__ void __launch_bounds__(256) weight_prep3d_kernel(const float* __restrict__ w, int Co, int Ci, int flip,
                                                            int out_major, T* out) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= Co * Ci * 27) return;
  const int t = e % 27, ci = (e / 27) % Ci, co = e / (27 * Ci);
  const int tp = flip ? 26 - t : t;
  const int o = flip ? ci : co, i = flip ? co : ci;
  const int O = flip ? Ci : Co, I = flip ? Co : Ci;
  const long dst = out_major ? ((long)tp * O + o) * I + i : ((long)tp * I + i) * O + o;
  out[dst] = Elt<T>::from_f(w[e]);
}

// every conv of a trunk (same shape) in one launch, both layouts: blockIdx.y = conv, the
// pointer tables travel in the kernel arguments (nothing to stage for graph capture)
constexpr int W3P_MAX = 16;
struct W3PrepMulti {
  const float* w[W3P_MAX];
  void* wk[W3P_MAX];
  void* wt[W3P_MAX];
};
template <typename T>
__global__ void __launch_bounds__(256) weight_prep3d_multi(W3PrepMulti m, int Co, int Ci, int out_major) {
  const int e = blockIdx.x * 256 + threadIdx.x;
  if (e >= Co * Ci * 27) return;
  const int c = blockIdx.y;
  const int t = e % 27, ci = (e / 27) % Ci, co = e / (27 * Ci);
  const T v = Elt<T>::from_f(m.w[c][e]);
  if (m.wk[c]) {
    const long dst = out_major ? ((long)t * Co + co) * Ci + ci : ((long)t * Ci + ci) * Co + co;
    reinterpret_cast<T*>(m.wk[c])[dst] = v;
  }
  if (m.wt[c]) {   // flipped taps, in / out exchanged
    const long dst = out_major ? ((long)(26 - t) * Ci + ci) * Co + co : ((long)(26 - t) * Co + co) * Ci + ci;
    reinterpret_cast<T*>(m.wt[c])[dst] = v;
  }
}

// depth split of the AFE mid_conv output: h [n][p][c * D + d] <-> x3 [n][d][p][c] (c = C)
template <typename T>
__global__ void __launch_bounds__(256) depth_split_kernel(const T* __restrict__ src, T* __restrict__ dst, int HW,
                                                          int C, int D, int inverse) {
  const long e = (long)blockIdx.x * 256 + threadIdx.x;   // index in x3 order
  const long tot = (long)gridDim.y * D * HW * C;
  (void)tot;
  const int n = blockIdx.y;
  const long per = (long)D * HW * C;
  if (e >= per) return;
  const int c = (int)(e % C), p = (int)((e / C) % HW), d = (int)(e / ((long)C * HW));
  const long i3 = (long)n * per + e;
  const long i2 = ((long)n * HW + p) * (C * D) + c * D + d;
  if (inverse) dst[i2] = src[i3];
  else dst[i3] = src[i2];
}

// bf16, C = 32, D = 16 (the AFE / Generator volume): one wave per 2 pixels, the 2 x 512-element
// [c][d] blocks through LDS -- every global access is a 32-B lane chunk (the element-wise kernel
// above reads 2 B per lane at a 32-B stride: 1.6 TB/s at B=8, r4 trace).  split: src
// [N][HW][c * 16 + d] -> dst [N][16][HW][32]; inverse: the reverse.
__global__ void __launch_bounds__(256) depth_split_c32d16(const bf16* __restrict__ src, bf16* __restrict__ dst,
                                                          int HW, int inverse) {
  __shared__ __attribute__((aligned(16))) bf16 sm[4][2 * 512];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const long pp = ((long)blockIdx.x * 4 + w) * 2;              // first of the wave's 2 pixels (n * HW + p)
  const int n = (int)(pp / HW), p0 = (int)(pp - (long)n * HW);
  bf16* const t = sm[w];
  // the lane's (pixel, d, 16-channel half) of the [N][16][HW][32] side
  const int px = lane >> 5, d = (lane & 31) >> 1, cb = (lane & 1) * 16;
  const long i3 = (((long)n * 16 + d) * HW + p0 + px) * 32 + cb;
  if (!inverse) {
    const uint4* s4 = reinterpret_cast<const uint4*>(src + pp * 512 + lane * 16);
    uint4* t4 = reinterpret_cast<uint4*>(t + lane * 16);
    t4[0] = s4[0];
    t4[1] = s4[1];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    bf16 v[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) v[k] = t[px * 512 + (cb + k) * 16 + d];
    uint4* o = reinterpret_cast<uint4*>(dst + i3);
    o[0] = *reinterpret_cast<const uint4*>(v);
    o[1] = *reinterpret_cast<const uint4*>(v + 8);
  } else {
    const uint4* s4 = reinterpret_cast<const uint4*>(src + i3);
    bf16 v[16];
    *reinterpret_cast<uint4*>(v) = s4[0];
    *reinterpret_cast<uint4*>(v + 8) = s4[1];
#pragma unroll
    for (int k = 0; k < 16; ++k) t[px * 512 + (cb + k) * 16 + d] = v[k];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    uint4* o = reinterpret_cast<uint4*>(dst + pp * 512 + lane * 16);
    const uint4* t4 = reinterpret_cast<const uint4*>(t + lane * 16);
    o[0] = t4[0];
    o[1] = t4[1];
  }
}

bool c32_fast(const fv_conv3d_desc* d) {
  return d->dtype == FV_BF16 && d->cin == 32 && d->cout == 32 && d->w == 64 && d->h % 4 == 0 &&
         (long)d->n * d->d * d->h * d->w * 32 * 2 < (1L << 31);
}

int check3(const fv_conv3d_desc* d) {
  FV_REQUIRE(d, "null conv3d descriptor");
  FV_REQUIRE(d->dtype == FV_F32 || d->dtype == FV_BF16, "conv3d dtype must be f32 or bf16");
  FV_REQUIRE(d->n > 0 && d->d > 0 && d->h > 0 && d->w > 0, "bad conv3d size");
  FV_REQUIRE(d->cin > 0 && d->cin <= 64 && d->cout > 0 && d->cout % 8 == 0,
             "conv3d: cin in 1..64, cout a multiple of 8");
  return FV_OK;
}

// conv3d_c32_fwd_dr walks dchunk + 2 input slices in peeled groups of three
bool c3r_chunk_ok(int dchunk) { return dchunk >= 4 && (dchunk + 2) % 3 == 0; }
// depth chunks per block for the forward kernels.  conv3d_c32_fwd_dr (one block per CU): the
// fewest chunks whose grid covers the 256 CUs, among the chunk lengths it walks, else the most;
// conv3d_c32_fwd when no chunk length fits: enough blocks to cover the CUs twice
int c3_ndc(const fv_conv3d_desc* d) {
  int best = 0;
  for (int k = 1; k <= d->d; k *= 2) {
    if (d->d % k || !c3r_chunk_ok(d->d / k)) continue;
    best = k;
    if ((long)d->n * (d->h / C3_TH) * k >= 256) break;
  }
  if (best) return best;
  int ndc = 1;
  while ((long)d->n * (d->h / C3_TH) * ndc < 512 && d->d % (2 * ndc) == 0 && d->d / (2 * ndc) >= 2) ndc *= 2;
  return ndc;
}
int c3w_nper(const fv_conv3d_desc* d) {
  const int nht = d->h / W3_TH;
  int nper = 1;
  while (d->n % (2 * nper) == 0 && (long)(d->n / (2 * nper)) * nht >= 256) nper *= 2;
  return nper;
}
// depth chunks: split the depth walk until the grid covers the 256 CUs (chunks of >= 4 slices;
// each chunk re-stages its 2 halo slices)
int c3w_ndc(const fv_conv3d_desc* d) {
  const long nb0 = (long)(d->n / c3w_nper(d)) * (d->h / W3_TH);
  int ndc = 1;
  while (nb0 * ndc < 256 && d->d / (2 * ndc) >= 4) ndc *= 2;
  return ndc;
}
int c3w_nblk(const fv_conv3d_desc* d) { return (d->n / c3w_nper(d)) * (d->h / W3_TH) * c3w_ndc(d); }
constexpr int C3W_NS = 16;

}  // namespace

extern "C" {

size_t fv_conv3d_wk_bytes(const fv_conv3d_desc* d) {
  if (check3(d)) return 0;
  return (size_t)27 * d->cin * d->cout * (c32_fast(d) ? 2 : 4);
}

int fv_conv3d_weight_prep(const fv_conv3d_desc* d, const float* w, void* wk, void* wt, void* stream) {
  int st = check3(d);
  if (st) return st;
  FV_REQUIRE(w, "null weight");
  hipStream_t s = (hipStream_t)stream;
  const int nb = fv_cdiv(27L * d->cin * d->cout, 256);
  // fast path: [t][out][in] bf16 (MFMA A fragments); direct path: [t][in][out] fp32
  const bool fast = c32_fast(d);
  if (wk) {
    if (fast) hipLaunchKernelGGL(weight_prep3d_kernel<bf16>, dim3(nb), dim3(256), 0, s, w, d->cout, d->cin, 0, 1, (bf16*)wk);
    else hipLaunchKernelGGL(weight_prep3d_kernel<float>, dim3(nb), dim3(256), 0, s, w, d->cout, d->cin, 0, 0, (float*)wk);
    if ((st = fv_check_launch("conv3d_weight_prep"))) return st;
  }
  if (wt) {
    if (fast) hipLaunchKernelGGL(weight_prep3d_kernel<bf16>, dim3(nb), dim3(256), 0, s, w, d->cout, d->cin, 1, 1, (bf16*)wt);
    else hipLaunchKernelGGL(weight_prep3d_kernel<float>, dim3(nb), dim3(256), 0, s, w, d->cout, d->cin, 1, 0, (float*)wt);
    if ((st = fv_check_launch("conv3d_weight_prep_t"))) return st;
  }
  return FV_OK;
}

int fv_conv3d_weight_prep_multi(const fv_conv3d_desc* d, int n, const float* const* w, void* const* wk,
                                void* const* wt, void* stream) {
  int st = check3(d);
  if (st) return st;
  FV_REQUIRE(n >= 0 && (n == 0 || (w && wk && wt)), "conv3d_weight_prep_multi: bad argument");
  hipStream_t s = (hipStream_t)stream;
  const bool fast = c32_fast(d);
  const int nb = fv_cdiv(27L * d->cin * d->cout, 256);
  for (int c0 = 0; c0 < n; c0 += W3P_MAX) {
    const int k = n - c0 < W3P_MAX ? n - c0 : W3P_MAX;
    W3PrepMulti m{};
    for (int c = 0; c < k; ++c) {
      FV_REQUIRE(w[c0 + c], "conv3d_weight_prep_multi: null weight");
      m.w[c] = w[c0 + c], m.wk[c] = wk[c0 + c], m.wt[c] = wt[c0 + c];
    }
    if (fast) hipLaunchKernelGGL(weight_prep3d_multi<bf16>, dim3(nb, k), dim3(256), 0, s, m, d->cout, d->cin, 1);
    else hipLaunchKernelGGL(weight_prep3d_multi<float>, dim3(nb, k), dim3(256), 0, s, m, d->cout, d->cin, 0);
    if ((st = fv_check_launch("conv3d_weight_prep_multi"))) return st;
  }
  return FV_OK;
}

int fv_conv3d_stats_blocks(const fv_conv3d_desc* d) {
  if (check3(d) || !c32_fast(d)) return 0;
  return d->n * (d->h / C3_TH) * c3_ndc(d) * C3_TH;
}
int fv_conv3d_stats_block_pixels(const fv_conv3d_desc* d) {
  if (check3(d) || !c32_fast(d)) return 0;
  return (d->d / c3_ndc(d)) * 64;
}

static int conv3d_run(const fv_conv3d_desc* d, int cin, int cout, const void* x, const void* w, const float* bias,
                      const void* res, void* y, float* stats, hipStream_t s) {
  if (c32_fast(d)) {
    C3Args a{};
    a.x = (const bf16*)x; a.w = (const bf16*)w; a.bias = bias; a.res = (const bf16*)res; a.y = (bf16*)y;
    a.stats = stats;
    a.N = d->n; a.D = d->d; a.H = d->h;
    a.ndc = c3_ndc(d);
    a.dchunk = d->d / a.ndc;
    a.xbytes = (unsigned)((long)d->n * d->d * d->h * 64 * 32 * 2);
    const int nblk = d->n * (d->h / C3_TH) * a.ndc;
    if (c3r_chunk_ok(a.dchunk)) {
      // the BN-partials and residual epilogue terms as compile-time switches (the data gradient
      // and the block's first conv skip their VALU / DMA)
      if (a.stats && a.res) hipLaunchKernelGGL((conv3d_c32_fwd_dr<true, true>), dim3(nblk), dim3(256), 0, s, a);
      else if (a.stats) hipLaunchKernelGGL((conv3d_c32_fwd_dr<true, false>), dim3(nblk), dim3(256), 0, s, a);
      else if (a.res) hipLaunchKernelGGL((conv3d_c32_fwd_dr<false, true>), dim3(nblk), dim3(256), 0, s, a);
      else hipLaunchKernelGGL((conv3d_c32_fwd_dr<false, false>), dim3(nblk), dim3(256), 0, s, a);
    }
    else hipLaunchKernelGGL((conv3d_c32_fwd<2>), dim3(nblk), dim3(256), 0, s, a);
    return fv_check_launch("conv3d_c32_fwd");
  }
  FV_REQUIRE(!stats, "conv3d: BN partials only on the fast path (query fv_conv3d_stats_blocks)");
  FV_REQUIRE(cout % 8 == 0, "conv3d: output channels must be a multiple of 8");
  const long V = (long)d->n * d->d * d->h * d->w;
  const long nthr = V * (cout / 8);
  if (d->dtype == FV_BF16)
    hipLaunchKernelGGL(conv3d_direct_fwd<bf16>, dim3(fv_cdiv(nthr, 256)), dim3(256), 0, s, (const bf16*)x,
                       (const float*)w, bias, (const bf16*)res, (bf16*)y, d->n, d->d, d->h, d->w, cin, cout);
  else
    hipLaunchKernelGGL(conv3d_direct_fwd<float>, dim3(fv_cdiv(nthr, 256)), dim3(256), 0, s, (const float*)x,
                       (const float*)w, bias, (const float*)res, (float*)y, d->n, d->d, d->h, d->w, cin, cout);
  return fv_check_launch("conv3d_direct");
}

int fv_conv3d_fwd(const fv_conv3d_desc* d, const void* x, const void* wk, const float* bias, const void* res,
                  void* y, float* stats, void* stream) {
  int st = check3(d);
  if (st) return st;
  FV_REQUIRE(x && wk && y, "null pointer");
  return conv3d_run(d, d->cin, d->cout, x, wk, bias, res, y, stats, (hipStream_t)stream);
}

int fv_conv3d_bwd_data(const fv_conv3d_desc* d, const void* dy, const void* wt, void* dx, void* stream) {
  int st = check3(d);
  if (st) return st;
  FV_REQUIRE(dy && wt && dx, "null pointer");
  FV_REQUIRE(d->cin % 8 == 0, "conv3d data gradient: cin must be a multiple of 8");
  return conv3d_run(d, d->cout, d->cin, dy, wt, nullptr, nullptr, dx, nullptr, (hipStream_t)stream);
}

size_t fv_conv3d_wgrad_ws_bytes(const fv_conv3d_desc* d) {
  if (check3(d) || !c32_fast(d)) return 0;
  return ((size_t)c3w_nblk(d) * (32 * 864 + 32) + (size_t)C3W_NS * (32 * 864 + 32)) * 4;
}

int fv_conv3d_bwd_weight(const fv_conv3d_desc* d, const void* x, const void* dy, float* dw, float* db, void* ws,
                         void* stream) {
  int st = check3(d);
  if (st) return st;
  FV_REQUIRE(x && dy && dw, "null pointer");
  hipStream_t s = (hipStream_t)stream;
  if (c32_fast(d)) {
    FV_REQUIRE(ws, "conv3d wgrad: workspace of fv_conv3d_wgrad_ws_bytes needed");
    const int nblk = c3w_nblk(d);
    C3WArgs a{};
    a.x = (const bf16*)x; a.dy = (const bf16*)dy;
    a.slab = (float*)ws;
    a.bslab = db ? a.slab + (long)nblk * 32 * 864 : nullptr;
    a.N = d->n; a.D = d->d; a.H = d->h; a.nper = c3w_nper(d); a.ndc = c3w_ndc(d);
    a.xbytes = a.dybytes = (unsigned)((long)d->n * d->d * d->h * 64 * 32 * 2);
    hipLaunchKernelGGL(conv3d_c32_wgrad, dim3(nblk), dim3(512), 0, s, a);
    if ((st = fv_check_launch("conv3d_c32_wgrad"))) return st;
    float* part = a.slab + (long)nblk * (32 * 864 + 32);
    const int ns = nblk < C3W_NS ? nblk : C3W_NS;
    hipLaunchKernelGGL(c3w_reduce1, dim3(fv_cdiv(32 * 864 + 32, 256), ns), dim3(256), 0, s, a.slab, a.bslab, nblk,
                       ns, part);
    if ((st = fv_check_launch("conv3d_wgrad_reduce1"))) return st;
    hipLaunchKernelGGL(c3w_reduce2, dim3(fv_cdiv(32 * 864 + 32, 256)), dim3(256), 0, s, part, ns, dw, db);
    return fv_check_launch("conv3d_wgrad_reduce2");
  }
  FV_REQUIRE(d->cin <= 64, "conv3d wgrad: cin <= 64");
  if (d->dtype == FV_BF16)
    hipLaunchKernelGGL(conv3d_direct_wgrad<bf16>, dim3(27 * d->cout), dim3(256), 0, s, (const bf16*)x,
                       (const bf16*)dy, dw, db, d->n, d->d, d->h, d->w, d->cin, d->cout);
  else
    hipLaunchKernelGGL(conv3d_direct_wgrad<float>, dim3(27 * d->cout), dim3(256), 0, s, (const float*)x,
                       (const float*)dy, dw, db, d->n, d->d, d->h, d->w, d->cin, d->cout);
  return fv_check_launch("conv3d_direct_wgrad");
}

int fv_depth_split(int dtype, const void* src, int n, int hw, int c, int d, int inverse, void* dst, void* stream) {
  FV_REQUIRE(src && dst && n > 0 && hw > 0 && c > 0 && d > 0, "depth_split: bad argument");
  FV_REQUIRE(dtype == FV_F32 || dtype == FV_BF16, "depth_split: f32 or bf16");
  const long per = (long)d * hw * c;
  if (dtype == FV_BF16 && c == 32 && d == 16 && ((long)n * hw) % 8 == 0) {
    hipLaunchKernelGGL(depth_split_c32d16, dim3((unsigned)((long)n * hw / 8)), dim3(256), 0, (hipStream_t)stream,
                       (const bf16*)src, (bf16*)dst, hw, inverse);
    return fv_check_launch("depth_split");
  }
  dim3 g(fv_cdiv(per, 256), n);
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(depth_split_kernel<bf16>, g, dim3(256), 0, (hipStream_t)stream, (const bf16*)src, (bf16*)dst,
                       hw, c, d, inverse);
  else
    hipLaunchKernelGGL(depth_split_kernel<float>, g, dim3(256), 0, (hipStream_t)stream, (const float*)src, (float*)dst,
                       hw, c, d, inverse);
  return fv_check_launch("depth_split");
}

}  // extern "C"
