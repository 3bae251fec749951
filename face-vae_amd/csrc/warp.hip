// Warp path of the Generator / MFE for gfx950: trilinear grid sampling, occlusion, and the
// MFE motion assembly.  All of it is HBM / gather bound (no MFMA): channels-last rows make
// every corner gather one contiguous row, lanes run along channels so the backward's
// scattered float atomics leave as whole 64-256 B row segments.
//
// Reference behaviour replaced (file:line in Luh1124/face-vae):
//   F.grid_sample(fs, deformation, align_corners=True) [trilinear, zeros]  models.py:1103
//   fs * occlusion                                                            models.py:1106
//   create_sparse_motions / create_heatmap_representations /
//   create_deformed_source_image (utils.py:139-179, kp2gaussian_3d 123-129,
//   make_coordinate_grid_3d 91-103), MFE mask softmax + deformation sum     models.py:1076-1078
#include "common.h"

namespace {

__device__ __forceinline__ float ld(const float* p) { return *p; }
__device__ __forceinline__ float ld(const bf16* p) { return (float)*p; }

// align_corners=True source index: ((g + 1) / 2) * (size - 1)
__device__ __forceinline__ float src_index(float g, int size) { return (g + 1.f) * 0.5f * (float)(size - 1); }

// lanes per voxel LPV (power of two <= 64), lane q of a voxel handles channels q, q + LPV, ...
template <typename T, int LPV>
__global__ void __launch_bounds__(256) grid_sample3d_fwd(const T* __restrict__ in, const float* __restrict__ grid,
                                                         T* __restrict__ out, int B, int Di, int Hi, int Wi, int Do,
                                                         int Ho, int Wo, int C, int group) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long v = gid / LPV;
  const int q = (int)(gid % LPV);
  const long Vo = (long)Do * Ho * Wo;
  if (v >= (long)B * Vo) return;
  const int b = (int)(v / Vo);
  const float* gp = grid + v * 3;
  const float ix = src_index(gp[0], Wi), iy = src_index(gp[1], Hi), iz = src_index(gp[2], Di);
  const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
  const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
  const float tx = ix - fx, ty = iy - fy, tz = iz - fz;
  const T* base = in + (long)(b / group) * Di * Hi * Wi * C;
  for (int c = q; c < C; c += LPV) {
    float acc = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
      const int xx = x0 + dx, yy = y0 + dy, zz = z0 + dz;
      if ((unsigned)xx < (unsigned)Wi && (unsigned)yy < (unsigned)Hi && (unsigned)zz < (unsigned)Di) {
        const float w = (dx ? tx : 1.f - tx) * (dy ? ty : 1.f - ty) * (dz ? tz : 1.f - tz);
        acc += w * ld(base + (((long)zz * Hi + yy) * Wi + xx) * C + c);
      }
    }
    out[v * C + c] = Elt<T>::from_f(acc);
  }
}

// backward: gin (fp32, zeroed, the input's layout) += w * gout by float atomics; ggrid per
// voxel = sum_c gout_c * d(out_c)/d(grid), reduced over the voxel's LPV lanes
template <typename T, int LPV>
__global__ void __launch_bounds__(256) grid_sample3d_bwd(const T* __restrict__ in, const float* __restrict__ grid,
                                                         const T* __restrict__ gout, float* gin, float* ggrid,
                                                         int B, int Di, int Hi, int Wi, int Do, int Ho, int Wo,
                                                         int C, int group) {
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long v = gid / LPV;
  const int q = (int)(gid % LPV);
  const long Vo = (long)Do * Ho * Wo;
  const bool live = v < (long)B * Vo;
  const long vv = live ? v : 0;
  const int b = (int)(vv / Vo);
  const float* gp = grid + vv * 3;
  const float ix = src_index(gp[0], Wi), iy = src_index(gp[1], Hi), iz = src_index(gp[2], Di);
  const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
  const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
  const float tx = ix - fx, ty = iy - fy, tz = iz - fz;
  const long boff = (long)(b / group) * Di * Hi * Wi * C;
  float gx = 0.f, gy = 0.f, gz = 0.f;
  if (live) {
    for (int c = q; c < C; c += LPV) {
      const float g = ld(gout + vv * C + c);
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
        const int xx = x0 + dx, yy = y0 + dy, zz = z0 + dz;
        if ((unsigned)xx < (unsigned)Wi && (unsigned)yy < (unsigned)Hi && (unsigned)zz < (unsigned)Di) {
          const float wx = dx ? tx : 1.f - tx, wy = dy ? ty : 1.f - ty, wz = dz ? tz : 1.f - tz;
          const long off = boff + (((long)zz * Hi + yy) * Wi + xx) * C + c;
          if (gin) atomicAdd(gin + off, wx * wy * wz * g);
          if (ggrid) {
            const float val = ld(in + off) * g;
            gx += (dx ? 1.f : -1.f) * wy * wz * val;
            gy += (dy ? 1.f : -1.f) * wx * wz * val;
            gz += (dz ? 1.f : -1.f) * wx * wy * val;
          }
        }
      }
    }
  }
  if (ggrid) {
#pragma unroll
    for (int o = 1; o < LPV; o <<= 1) {
      gx += __shfl_xor(gx, o, 64);
      gy += __shfl_xor(gy, o, 64);
      gz += __shfl_xor(gz, o, 64);
    }
    if (live && q == 0) {
      ggrid[vv * 3 + 0] = gx * 0.5f * (float)(Wi - 1);
      ggrid[vv * 3 + 1] = gy * 0.5f * (float)(Hi - 1);
      ggrid[vv * 3 + 2] = gz * 0.5f * (float)(Di - 1);
    }
  }
}

// forward with lanes over 8-channel chunks (Chunk8: 16 B bf16 / 32 B fp32 per corner gather;
// C % 8 == 0): the 1-channel-per-lane kernel above issued eight 2-byte gathers per bf16 row of
// 64 B.  Same corner order and arithmetic -> bit-identical.
template <typename T>
__global__ void __launch_bounds__(256) grid_sample3d_fwd8(const T* __restrict__ in, const float* __restrict__ grid,
                                                          T* __restrict__ out, int B, int Di, int Hi, int Wi, long Vo,
                                                          int C, int group) {
  const int C8 = C >> 3;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long v = gid / C8;
  const int q = (int)(gid - v * C8);
  if (v >= (long)B * Vo) return;
  const int b = (int)(v / Vo);
  const float* gp = grid + v * 3;
  const float ix = src_index(gp[0], Wi), iy = src_index(gp[1], Hi), iz = src_index(gp[2], Di);
  const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
  const int x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
  const float tx = ix - fx, ty = iy - fy, tz = iz - fz;
  const T* base = in + (long)(b / group) * Di * Hi * Wi * C + q * 8;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
    const int xx = x0 + dx, yy = y0 + dy, zz = z0 + dz;
    if ((unsigned)xx < (unsigned)Wi && (unsigned)yy < (unsigned)Hi && (unsigned)zz < (unsigned)Di) {
      const float w = (dx ? tx : 1.f - tx) * (dy ? ty : 1.f - ty) * (dz ? tz : 1.f - tz);
      Chunk8<T> c;
      c.load(base + (((long)zz * Hi + yy) * Wi + xx) * C);
#pragma unroll
      for (int j = 0; j < 8; ++j) acc[j] += w * c.get(j);
    }
  }
  Chunk8<T> o;
  o.set8(acc);
  o.store(out + v * C + q * 8);
}

// ---- input gradient by gathering (fv_grid_sample3d_bwd_input) --------------------------------
// The scatter above adds 8 corners x C float atomics per output voxel (134 M at the §8(f) shape,
// 395 µs at B = 8).  Instead: bucket the output voxels by their base input cell (x0, y0, z0) --
// one int atomic per voxel for the counts, an exclusive scan, a fill -- and let each input cell
// sum the up-to-8 buckets whose corner it is.  Every gin element is written once, no zeroing.
// Bucket keys cover base cells in [-1, size - 1] per axis (a voxel whose base is outside has no
// corner inside and drops out).
struct GsRec {
  int v;
  float tx, ty, tz;
};
constexpr int GS_SCAN = 1024;   // counts per scan block

__device__ __forceinline__ bool gs_base(const float* grid, long v, int Di, int Hi, int Wi, int& x0, int& y0, int& z0,
                                        float& tx, float& ty, float& tz) {
  const float* gp = grid + v * 3;
  const float ix = src_index(gp[0], Wi), iy = src_index(gp[1], Hi), iz = src_index(gp[2], Di);
  const float fx = floorf(ix), fy = floorf(iy), fz = floorf(iz);
  // NaN and far-outside coordinates fail these tests before any float -> int conversion
  if (!(fx >= -1.f && fx <= (float)(Wi - 1) && fy >= -1.f && fy <= (float)(Hi - 1) && fz >= -1.f &&
        fz <= (float)(Di - 1)))
    return false;
  x0 = (int)fx, y0 = (int)fy, z0 = (int)fz;
  tx = ix - fx, ty = iy - fy, tz = iz - fz;
  return true;
}
__device__ __forceinline__ int gs_key(int bi, int z0, int y0, int x0, int Di, int Hi, int Wi) {
  return ((bi * (Di + 1) + z0 + 1) * (Hi + 1) + y0 + 1) * (Wi + 1) + x0 + 1;
}

__global__ void __launch_bounds__(256) gs_bucket_count(const float* __restrict__ grid, long nvox, long Vo, int Di,
                                                       int Hi, int Wi, int group, int* __restrict__ cnt,
                                                       int2* __restrict__ keyrank) {
  const long v = (long)blockIdx.x * 256 + threadIdx.x;
  if (v >= nvox) return;
  int x0, y0, z0;
  float tx, ty, tz;
  int2 kr = make_int2(-1, 0);
  if (gs_base(grid, v, Di, Hi, Wi, x0, y0, z0, tx, ty, tz)) {
    kr.x = gs_key((int)(v / Vo) / group, z0, y0, x0, Di, Hi, Wi);
    kr.y = atomicAdd(cnt + kr.x, 1);
  }
  keyrank[v] = kr;
}

// exclusive scan of the block's 1024 values a[4] per thread; returns the thread's prefix and the
// block total in *total (256 threads)
__device__ __forceinline__ int gs_block_scan(const int (&a)[4], int* total) {
  __shared__ int wsum[4];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int t = a[0] + a[1] + a[2] + a[3];
  int x = t;
#pragma unroll
  for (int o = 1; o < 64; o <<= 1) {
    const int y = __shfl_up(x, o, 64);
    if (lane >= o) x += y;
  }
  if (lane == 63) wsum[w] = x;
  __syncthreads();
  int wo = 0;
#pragma unroll
  for (int k = 0; k < 4; ++k) wo += k < w ? wsum[k] : 0;
  *total = wsum[0] + wsum[1] + wsum[2] + wsum[3];
  __syncthreads();
  return wo + x - t;
}

// cnt[0, n) -> offsets within each 1024-block; bsum[blk] = the block's total
__global__ void __launch_bounds__(256) gs_scan_blocks(int* __restrict__ cnt, long n, int* __restrict__ bsum) {
  const long i0 = (long)blockIdx.x * GS_SCAN + threadIdx.x * 4;
  int a[4];
#pragma unroll
  for (int j = 0; j < 4; ++j) a[j] = i0 + j < n ? cnt[i0 + j] : 0;
  int total;
  int e = gs_block_scan(a, &total);
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    if (i0 + j < n) cnt[i0 + j] = e;
    e += a[j];
  }
  if (threadIdx.x == 0) bsum[blockIdx.x] = total;
}

// one block: bsum[0, nb) -> exclusive prefix sums, 1024 at a time with a carry
__global__ void __launch_bounds__(256) gs_scan_totals(int* __restrict__ bsum, int nb, int* __restrict__ lst) {
  if (threadIdx.x == 0) lst[0] = 0, lst[1] = 0;
  int carry = 0;
  for (int base = 0; base < nb; base += GS_SCAN) {
    const int i0 = base + threadIdx.x * 4;
    int a[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) a[j] = i0 + j < nb ? bsum[i0 + j] : 0;
    int total;
    int e = gs_block_scan(a, &total) + carry;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      if (i0 + j < nb) bsum[i0 + j] = e;
      e += a[j];
    }
    carry += total;
  }
}

__device__ __forceinline__ int gs_offset(const int* off, const int* boff, int key) {
  return off[key] + boff[key / GS_SCAN];
}

__global__ void __launch_bounds__(256) gs_bucket_fill(const float* __restrict__ grid, const int2* __restrict__ keyrank,
                                                      const int* __restrict__ off, const int* __restrict__ boff,
                                                      long nvox, int Di, int Hi, int Wi, GsRec* __restrict__ rec) {
  const long v = (long)blockIdx.x * 256 + threadIdx.x;
  if (v >= nvox) return;
  const int2 kr = keyrank[v];
  if (kr.x < 0) return;
  int x0, y0, z0;
  float tx, ty, tz;
  gs_base(grid, v, Di, Hi, Wi, x0, y0, z0, tx, ty, tz);
  GsRec r;
  r.v = (int)v, r.tx = tx, r.ty = ty, r.tz = tz;
  rec[gs_offset(off, boff, kr.x) + kr.y] = r;
}

// The fill places a bucket's records in atomicAdd-rank order, which changes run to run; the
// gather sums them in bucket order, so every bucket is put in voxel-index order and the input
// gradient is bit-reproducible.  No lane sorts more than GS_INS records alone: one thread per
// bucket insertion-sorts the common few and appends the larger buckets' keys to two lists
// (wave-aggregated), which gs_bucket_sort_coop works through with whole workgroups -- a bitonic
// sort in LDS up to GS_MID records, and above that (a degenerate or collapsed motion grid piling
// voxels onto one cell) a stable compaction: the workgroup streams keyrank in voxel order and
// re-emits the bucket's records in that order, O(nvox / 1024) block steps per big bucket instead
// of one lane's O(n log n) walk through global memory.
constexpr int GS_INS = 16, GS_MID = 2048, GS_COOP_BLOCKS = 256;

__device__ __forceinline__ void gs_append(bool p, int* ctr, int* list, int val) {
  const unsigned long long m = __ballot(p);
  if (!m) return;
  const int lane = threadIdx.x & 63, leader = __ffsll((long long)m) - 1;
  int base = 0;
  if (lane == leader) base = atomicAdd(ctr, __popcll(m));
  base = __shfl(base, leader, 64);
  if (p) list[base + __popcll(m & ((1ull << lane) - 1))] = val;
}

// lst[0] / lst[1]: counts of the mid / big lists (zeroed by gs_scan_totals), midk / bigk: keys
__global__ void __launch_bounds__(256) gs_bucket_sort(GsRec* __restrict__ rec, const int* __restrict__ off,
                                                      const int* __restrict__ boff, long nkey, int* __restrict__ lst,
                                                      int* __restrict__ midk, int* __restrict__ bigk) {
  const long key = (long)blockIdx.x * 256 + threadIdx.x;
  int b = 0, n = 0;
  if (key < nkey - 1) {
    b = gs_offset(off, boff, (int)key);
    n = gs_offset(off, boff, (int)key + 1) - b;
  }
  gs_append(n > GS_INS && n <= GS_MID, lst, midk, (int)key);
  gs_append(n > GS_MID, lst + 1, bigk, (int)key);
  if (n < 2 || n > GS_INS) return;
  GsRec* a = rec + b;
  for (int i = 1; i < n; ++i) {
    const GsRec x = a[i];
    int j = i - 1;
    while (j >= 0 && a[j].v > x.v) {
      a[j + 1] = a[j];
      --j;
    }
    a[j + 1] = x;
  }
}

// persistent over the two lists (GS_COOP_BLOCKS workgroups; every block exits once both are done)
__global__ void __launch_bounds__(256) gs_bucket_sort_coop(const float* __restrict__ grid,
                                                           const int2* __restrict__ keyrank, GsRec* __restrict__ rec,
                                                           const int* __restrict__ off, const int* __restrict__ boff,
                                                           const int* __restrict__ lst, const int* __restrict__ midk,
                                                           const int* __restrict__ bigk, long nvox, int Di, int Hi,
                                                           int Wi) {
  __shared__ GsRec s[GS_MID];
  const int tid = threadIdx.x;
  const int nmid = lst[0], nbig = lst[1];
  for (int i = blockIdx.x; i < nmid; i += gridDim.x) {
    const int key = midk[i];
    const int b = gs_offset(off, boff, key), n = gs_offset(off, boff, key + 1) - b;
    int P = 32;
    while (P < n) P <<= 1;
    for (int j = tid; j < P; j += 256) {
      if (j < n) s[j] = rec[b + j];
      else s[j].v = 0x7fffffff;
    }
    __syncthreads();
    for (int k = 2; k <= P; k <<= 1)
      for (int j = k >> 1; j > 0; j >>= 1) {
        for (int t = tid; t < P / 2; t += 256) {
          const int lo = 2 * t - (t & (j - 1)), hi = lo + j;
          const GsRec x = s[lo], y = s[hi];
          if ((x.v > y.v) == ((lo & k) == 0)) s[lo] = y, s[hi] = x;
        }
        __syncthreads();
      }
    for (int j = tid; j < n; j += 256) rec[b + j] = s[j];
    __syncthreads();
  }
  for (int i = blockIdx.x; i < nbig; i += gridDim.x) {
    const int key = bigk[i];
    GsRec* a = rec + gs_offset(off, boff, key);
    int run = 0;
    for (long v0 = 0; v0 < nvox; v0 += 1024) {
      int m[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const long v = v0 + tid * 4 + j;
        m[j] = v < nvox && keyrank[v].x == key;
      }
      int total;
      int e = gs_block_scan(m, &total) + run;
#pragma unroll
      for (int j = 0; j < 4; ++j)
        if (m[j]) {
          const long v = v0 + tid * 4 + j;
          int x0, y0, z0;
          GsRec r;
          gs_base(grid, v, Di, Hi, Wi, x0, y0, z0, r.tx, r.ty, r.tz);
          r.v = (int)v;
          a[e++] = r;
        }
      run += total;
    }
  }
}

// one lane per (input cell, V-channel chunk); V = 8 (Chunk8 rows, C % 8 == 0) or 1
template <typename T, int V>
__global__ void __launch_bounds__(256) gs_gather_input(const GsRec* __restrict__ rec, const int* __restrict__ off,
                                                       const int* __restrict__ boff, const T* __restrict__ gout,
                                                       long ncell, int Di, int Hi, int Wi, int C, T* __restrict__ gin) {
  const int CV = C / V;
  const long gid = (long)blockIdx.x * 256 + threadIdx.x;
  const long cell = gid / CV;
  const int q = (int)(gid - cell * CV);
  if (cell >= ncell) return;
  const int x = (int)(cell % Wi);
  long t = cell / Wi;
  const int y = (int)(t % Hi);
  t /= Hi;
  const int z = (int)(t % Di), bi = (int)(t / Di);
  float acc[V];
#pragma unroll
  for (int j = 0; j < V; ++j) acc[j] = 0.f;
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    const int dx = k & 1, dy = (k >> 1) & 1, dz = k >> 2;
    const int key = gs_key(bi, z - dz, y - dy, x - dx, Di, Hi, Wi);
    const int e = gs_offset(off, boff, key + 1);
    int r = gs_offset(off, boff, key);
    // long buckets (a collapsed motion grid piles many voxels onto one cell): four records'
    // loads in flight per step instead of one dependent pair, still summed in record order
    for (; e - r >= 8; r += 4) {
      GsRec R4[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) R4[u] = rec[r + u];
      if constexpr (V % 8 == 0) {
        Chunk8<T> c4[4][V / 8];
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
          for (int h = 0; h < V / 8; ++h) c4[u][h].load(gout + (long)R4[u].v * C + q * V + 8 * h);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const GsRec& R = R4[u];
          const float w = (dx ? R.tx : 1.f - R.tx) * (dy ? R.ty : 1.f - R.ty) * (dz ? R.tz : 1.f - R.tz);
#pragma unroll
          for (int h = 0; h < V / 8; ++h)
#pragma unroll
            for (int j = 0; j < 8; ++j) acc[8 * h + j] += w * c4[u][h].get(j);
        }
      } else {
        float g4[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) g4[u] = ld(gout + (long)R4[u].v * C + q * V);
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const GsRec& R = R4[u];
          const float w = (dx ? R.tx : 1.f - R.tx) * (dy ? R.ty : 1.f - R.ty) * (dz ? R.tz : 1.f - R.tz);
          acc[0] += w * g4[u];
        }
      }
    }
    for (; r < e; ++r) {
      const GsRec R = rec[r];
      const float w = (dx ? R.tx : 1.f - R.tx) * (dy ? R.ty : 1.f - R.ty) * (dz ? R.tz : 1.f - R.tz);
      const T* g = gout + (long)R.v * C + q * V;
      if constexpr (V % 8 == 0) {
#pragma unroll
        for (int h = 0; h < V / 8; ++h) {
          Chunk8<T> c;
          c.load(g + 8 * h);
#pragma unroll
          for (int j = 0; j < 8; ++j) acc[8 * h + j] += w * c.get(j);
        }
      } else {
        acc[0] += w * ld(g);
      }
    }
  }
  T* o = gin + cell * C + q * V;
  if constexpr (V % 8 == 0) {
#pragma unroll
    for (int h = 0; h < V / 8; ++h) {
      Chunk8<T> c;
      c.set8(acc + 8 * h);
      c.store(o + 8 * h);
    }
  } else {
    o[0] = Elt<T>::from_f(acc[0]);
  }
}

struct GsWs {
  int *cnt, *bsum, *lst, *midk, *bigk;   // lst: the two list counts of gs_bucket_sort
  int2* keyrank;
  GsRec* rec;
  long nkey, nblk, nvox;
  size_t bytes;
};
static GsWs gs_ws_layout(void* base, int B, int Di, int Hi, int Wi, int Do, int Ho, int Wo, int group) {
  GsWs w;
  w.nvox = (long)B * Do * Ho * Wo;
  w.nkey = (long)(B / group) * (Di + 1) * (Hi + 1) * (Wi + 1) + 1;   // + 1: the end offset of the last key
  w.nblk = (w.nkey + GS_SCAN - 1) / GS_SCAN;
  auto up = [](size_t b) { return (b + 255) & ~(size_t)255; };
  char* p = (char*)base;
  size_t o = 0;
  w.cnt = (int*)(p + o), o += up(w.nkey * 4);
  w.bsum = (int*)(p + o), o += up(w.nblk * 4);
  w.keyrank = (int2*)(p + o), o += up(w.nvox * 8);
  w.rec = (GsRec*)(p + o), o += up(w.nvox * sizeof(GsRec));
  w.lst = (int*)(p + o), o += up(2 * 4);
  w.midk = (int*)(p + o), o += up((w.nvox / (GS_INS + 1) + 1) * 4);
  w.bigk = (int*)(p + o), o += up((w.nvox / (GS_MID + 1) + 1) * 4);
  w.bytes = o;
  return w;
}

template <typename T>
__global__ void __launch_bounds__(256) f32_to_kernel(const float* __restrict__ a, T* __restrict__ b, long n) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i < n) b[i] = Elt<T>::from_f(a[i]);
}

// occlusion: y[p][c] = x[p][c] * occ[p]; one wave per pixel (lanes along channels)
template <typename T>
__global__ void __launch_bounds__(256) occlusion_fwd(const T* __restrict__ x, const float* __restrict__ occ,
                                                     T* __restrict__ y, long P, int C) {
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const float o = occ[p];
  for (int c = threadIdx.x & 63; c < C; c += 64) y[p * C + c] = Elt<T>::from_f(ld(x + p * C + c) * o);
}
template <typename T>
__global__ void __launch_bounds__(256) occlusion_bwd(const T* __restrict__ g, const T* __restrict__ x,
                                                     const float* __restrict__ occ, T* dx, float* docc, long P,
                                                     int C) {
  const long p = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (p >= P) return;
  const float o = occ[p];
  float s = 0.f;
  for (int c = threadIdx.x & 63; c < C; c += 64) {
    const float gv = ld(g + p * C + c);
    if (dx) dx[p * C + c] = Elt<T>::from_f(gv * o);
    s += gv * ld(x + p * C + c);
  }
  s = wave_sum(s);
  if (docc && (threadIdx.x & 63) == 0) docc[p] = s;
}

// make_coordinate_grid_3d (utils.py:91-103): (x over W, y over H, z over D) in [-1, 1]
__device__ __forceinline__ void ident(long v, int D, int H, int W, float& gx, float& gy, float& gz) {
  const int w = (int)(v % W), h = (int)((v / W) % H), d = (int)(v / ((long)W * H));
  gx = 2.f * ((float)w / (float)(W - 1)) - 1.f;
  gy = 2.f * ((float)h / (float)(H - 1)) - 1.f;
  gz = 2.f * ((float)d / (float)(D - 1)) - 1.f;
}

// create_sparse_motions (utils.py:139-152): out[n][0] = identity, out[n][k+1] = J (id - kp_d[k]) + kp_s[k]
__global__ void __launch_bounds__(256) sparse_motion_fwd(const float* __restrict__ kps, const float* __restrict__ kpd,
                                                         const float* __restrict__ J, float* __restrict__ out, int N,
                                                         int K, int D, int H, int W) {
  const long V = (long)D * H * W;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * (K + 1) * V) return;
  const long v = i % V;
  const int k = (int)((i / V) % (K + 1)), n = (int)(i / (V * (K + 1)));
  float gx, gy, gz;
  ident(v, D, H, W, gx, gy, gz);
  float* o = out + i * 3;
  if (k == 0) {
    o[0] = gx; o[1] = gy; o[2] = gz;
    return;
  }
  const float* kd = kpd + ((long)n * K + k - 1) * 3;
  const float* ks = kps + ((long)n * K + k - 1) * 3;
  const float* j = J + (long)n * 9;
  const float c0 = gx - kd[0], c1 = gy - kd[1], c2 = gz - kd[2];
  o[0] = j[0] * c0 + j[1] * c1 + j[2] * c2 + ks[0];
  o[1] = j[3] * c0 + j[4] * c1 + j[5] * c2 + ks[1];
  o[2] = j[6] * c0 + j[7] * c1 + j[8] * c2 + ks[2];
}

// per (n, k >= 1): sums over voxels of g (3) and g (x) c (9), c = id - kp_d; block reduction
__global__ void __launch_bounds__(256) sparse_motion_bwd(const float* __restrict__ g, const float* __restrict__ kpd,
                                                         float* __restrict__ sums, int N, int K, int D, int H, int W) {
  const int k = blockIdx.x % K, n = blockIdx.x / K;
  const long V = (long)D * H * W;
  const float* gk = g + (((long)n * (K + 1) + k + 1) * V) * 3;
  const float* kd = kpd + ((long)n * K + k) * 3;
  float s[12];
#pragma unroll
  for (int j = 0; j < 12; ++j) s[j] = 0.f;
  for (long v = threadIdx.x; v < V; v += 256) {
    float gx, gy, gz;
    ident(v, D, H, W, gx, gy, gz);
    const float c[3] = {gx - kd[0], gy - kd[1], gz - kd[2]};
    const float gg[3] = {gk[v * 3], gk[v * 3 + 1], gk[v * 3 + 2]};
#pragma unroll
    for (int a = 0; a < 3; ++a) {
      s[a] += gg[a];
#pragma unroll
      for (int b = 0; b < 3; ++b) s[3 + 3 * a + b] += gg[a] * c[b];
    }
  }
  __shared__ float red[4][12];
#pragma unroll
  for (int j = 0; j < 12; ++j) {
    const float t = wave_sum(s[j]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][j] = t;
  }
  __syncthreads();
  if (threadIdx.x < 12) sums[(long)blockIdx.x * 12 + threadIdx.x] =
      red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
}

// create_heatmap_representations (utils.py:130-137 with kp2gaussian_3d 123-129):
// out[n][0] = 0, out[n][k+1] = G(kp_d[k]) - G(kp_s[k]), G(kp) = exp(-0.5 |id - kp|^2 / var)
__device__ __forceinline__ float gauss(float gx, float gy, float gz, const float* kp, float var) {
  const float a = gx - kp[0], b = gy - kp[1], c = gz - kp[2];
  return expf(-0.5f * (a * a + b * b + c * c) / var);
}
__global__ void __launch_bounds__(256) heatmap_fwd(const float* __restrict__ kps, const float* __restrict__ kpd,
                                                   float* __restrict__ out, int N, int K, int D, int H, int W,
                                                   float var) {
  const long V = (long)D * H * W;
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * (K + 1) * V) return;
  const long v = i % V;
  const int k = (int)((i / V) % (K + 1)), n = (int)(i / (V * (K + 1)));
  if (k == 0) {
    out[i] = 0.f;
    return;
  }
  float gx, gy, gz;
  ident(v, D, H, W, gx, gy, gz);
  out[i] = gauss(gx, gy, gz, kpd + ((long)n * K + k - 1) * 3, var) - gauss(gx, gy, gz, kps + ((long)n * K + k - 1) * 3, var);
}
// per (n, k): dkp_d = sum_v g G_d (id - kp_d) / var, dkp_s = -sum_v g G_s (id - kp_s) / var
__global__ void __launch_bounds__(256) heatmap_bwd(const float* __restrict__ g, const float* __restrict__ kps,
                                                   const float* __restrict__ kpd, float* dkps, float* dkpd, int N,
                                                   int K, int D, int H, int W, float var) {
  const int k = blockIdx.x % K, n = blockIdx.x / K;
  const long V = (long)D * H * W;
  const float* gk = g + ((long)n * (K + 1) + k + 1) * V;
  const float* pd = kpd + ((long)n * K + k) * 3;
  const float* ps = kps + ((long)n * K + k) * 3;
  float s[6] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (long v = threadIdx.x; v < V; v += 256) {
    float gx, gy, gz;
    ident(v, D, H, W, gx, gy, gz);
    const float gv = gk[v];
    const float ed = gv * gauss(gx, gy, gz, pd, var) / var, es = gv * gauss(gx, gy, gz, ps, var) / var;
    s[0] += ed * (gx - pd[0]);
    s[1] += ed * (gy - pd[1]);
    s[2] += ed * (gz - pd[2]);
    s[3] -= es * (gx - ps[0]);
    s[4] -= es * (gy - ps[1]);
    s[5] -= es * (gz - ps[2]);
  }
  __shared__ float red[4][6];
#pragma unroll
  for (int j = 0; j < 6; ++j) {
    const float t = wave_sum(s[j]);
    if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6][j] = t;
  }
  __syncthreads();
  if (threadIdx.x < 6) {
    const float t = red[0][threadIdx.x] + red[1][threadIdx.x] + red[2][threadIdx.x] + red[3][threadIdx.x];
    if (threadIdx.x < 3) dkpd[((long)n * K + k) * 3 + threadIdx.x] = t;
    else dkps[((long)n * K + k) * 3 + threadIdx.x - 3] = t;
  }
}

// MFE (models.py:1076-1078): p = softmax_k(logits[n][k][v]); def[n][v] = sum_k p_k sm[n][k][v]
__global__ void __launch_bounds__(256) motion_mask_fwd(const float* __restrict__ logits, const float* __restrict__ sm,
                                                       float* __restrict__ prob, float* __restrict__ def, int N,
                                                       int K1, long V) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * V) return;
  const long v = i % V;
  const int n = (int)(i / V);
  const float* l = logits + (long)n * K1 * V + v;
  float m = -INFINITY;
  for (int k = 0; k < K1; ++k) m = fmaxf(m, l[(long)k * V]);
  float z = 0.f;
  for (int k = 0; k < K1; ++k) z += expf(l[(long)k * V] - m);
  const float iz = 1.f / z;
  float d0 = 0.f, d1 = 0.f, d2 = 0.f;
  for (int k = 0; k < K1; ++k) {
    const float p = expf(l[(long)k * V] - m) * iz;
    if (prob) prob[((long)n * K1 + k) * V + v] = p;
    const float* s = sm + (((long)n * K1 + k) * V + v) * 3;
    d0 += p * s[0];
    d1 += p * s[1];
    d2 += p * s[2];
  }
  def[i * 3] = d0;
  def[i * 3 + 1] = d1;
  def[i * 3 + 2] = d2;
}
// backward: dsm = p g_def; dlogit_k = p_k (s_k - sum_j p_j s_j), s_k = g_def . sm_k + g_prob_k
__global__ void __launch_bounds__(256) motion_mask_bwd(const float* __restrict__ prob, const float* __restrict__ sm,
                                                       const float* __restrict__ gdef, const float* gprob,
                                                       float* dlogits, float* dsm, int N, int K1, long V) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;
  if (i >= (long)N * V) return;
  const long v = i % V;
  const int n = (int)(i / V);
  const float g0 = gdef[i * 3], g1 = gdef[i * 3 + 1], g2 = gdef[i * 3 + 2];
  float ps = 0.f;
  for (int k = 0; k < K1; ++k) {
    const long e = ((long)n * K1 + k) * V + v;
    const float p = prob[e];
    const float* s = sm + e * 3;
    const float sk = g0 * s[0] + g1 * s[1] + g2 * s[2] + (gprob ? gprob[e] : 0.f);
    ps += p * sk;
    if (dsm) {
      dsm[e * 3] = p * g0;
      dsm[e * 3 + 1] = p * g1;
      dsm[e * 3 + 2] = p * g2;
    }
  }
  if (dlogits) {
    for (int k = 0; k < K1; ++k) {
      const long e = ((long)n * K1 + k) * V + v;
      const float* s = sm + e * 3;
      const float sk = g0 * s[0] + g1 * s[1] + g2 * s[2] + (gprob ? gprob[e] : 0.f);
      dlogits[e] = prob[e] * (sk - ps);
    }
  }
}

int lpv_of(int C) {
  int l = 1;
  while (l < C && l < 64) l <<= 1;
  return l;
}

}  // namespace

extern "C" {

int fv_grid_sample3d_fwd(int dtype, const void* in, const float* grid, int B, int Di, int Hi, int Wi, int Do,
                         int Ho, int Wo, int C, int group, void* out, void* stream) {
  FV_REQUIRE(in && grid && out && B > 0 && C > 0 && group > 0 && B % group == 0, "grid_sample3d: bad argument");
  FV_REQUIRE(dtype == FV_F32 || dtype == FV_BF16, "grid_sample3d: f32 or bf16");
  hipStream_t s = (hipStream_t)stream;
  const long nvox = (long)B * Do * Ho * Wo;
  if (C % 8 == 0) {
    const int nb8 = fv_cdiv(nvox * (C / 8), 256);
    if (dtype == FV_BF16)
      hipLaunchKernelGGL(grid_sample3d_fwd8<bf16>, dim3(nb8), dim3(256), 0, s, (const bf16*)in, grid, (bf16*)out, B,
                         Di, Hi, Wi, (long)Do * Ho * Wo, C, group);
    else
      hipLaunchKernelGGL(grid_sample3d_fwd8<float>, dim3(nb8), dim3(256), 0, s, (const float*)in, grid, (float*)out,
                         B, Di, Hi, Wi, (long)Do * Ho * Wo, C, group);
    return fv_check_launch("grid_sample3d_fwd");
  }
  const int lpv = lpv_of(C);
  const int nb = fv_cdiv(nvox * lpv, 256);
#define GS_FWD(T, L)                                                                                              \
  hipLaunchKernelGGL((grid_sample3d_fwd<T, L>), dim3(nb), dim3(256), 0, s, (const T*)in, grid, (T*)out, B, Di, Hi, \
                     Wi, Do, Ho, Wo, C, group)
#define GS_DISPATCH(M, T)               \
  switch (lpv) {                        \
    case 1: M(T, 1); break;             \
    case 2: M(T, 2); break;             \
    case 4: M(T, 4); break;             \
    case 8: M(T, 8); break;             \
    case 16: M(T, 16); break;           \
    case 32: M(T, 32); break;           \
    default: M(T, 64); break;           \
  }
  if (dtype == FV_BF16) {
    GS_DISPATCH(GS_FWD, bf16)
  } else {
    GS_DISPATCH(GS_FWD, float)
  }
  return fv_check_launch("grid_sample3d_fwd");
}

/* gin: fp32 accumulation buffer in the input's layout, zeroed by the caller (may be NULL);
 * ggrid: [B][Do][Ho][Wo][3] fp32 (may be NULL) */
int fv_grid_sample3d_bwd(int dtype, const void* in, const float* grid, const void* gout, int B, int Di, int Hi,
                         int Wi, int Do, int Ho, int Wo, int C, int group, float* gin, float* ggrid, void* stream) {
  FV_REQUIRE(in && grid && gout && B > 0 && C > 0 && group > 0 && B % group == 0, "grid_sample3d_bwd: bad argument");
  FV_REQUIRE(dtype == FV_F32 || dtype == FV_BF16, "grid_sample3d: f32 or bf16");
  hipStream_t s = (hipStream_t)stream;
  const long nvox = (long)B * Do * Ho * Wo;
  const int lpv = lpv_of(C);
  const int nb = fv_cdiv(nvox * lpv, 256);
#define GS_BWD(T, L)                                                                                              \
  hipLaunchKernelGGL((grid_sample3d_bwd<T, L>), dim3(nb), dim3(256), 0, s, (const T*)in, grid, (const T*)gout, gin, \
                     ggrid, B, Di, Hi, Wi, Do, Ho, Wo, C, group)
  if (dtype == FV_BF16) {
    GS_DISPATCH(GS_BWD, bf16)
  } else {
    GS_DISPATCH(GS_BWD, float)
  }
  return fv_check_launch("grid_sample3d_bwd");
}

size_t fv_grid_sample3d_bwd_input_ws_bytes(int B, int Di, int Hi, int Wi, int Do, int Ho, int Wo, int group) {
  if (B <= 0 || group <= 0 || B % group) return 0;
  return gs_ws_layout(nullptr, B, Di, Hi, Wi, Do, Ho, Wo, group).bytes;
}

int fv_grid_sample3d_bwd_input(int dtype, const float* grid, const void* gout, int B, int Di, int Hi, int Wi, int Do,
                               int Ho, int Wo, int C, int group, void* gin, void* ws, void* stream) {
  FV_REQUIRE(grid && gout && gin && ws && B > 0 && C > 0 && group > 0 && B % group == 0 && Di > 0 && Hi > 0 &&
                 Wi > 0 && Do > 0 && Ho > 0 && Wo > 0,
             "grid_sample3d_bwd_input: bad argument");
  FV_REQUIRE(dtype == FV_F32 || dtype == FV_BF16, "grid_sample3d_bwd_input: f32 or bf16");
  const GsWs w = gs_ws_layout(ws, B, Di, Hi, Wi, Do, Ho, Wo, group);
  FV_REQUIRE(w.nvox < (1L << 31) && w.nkey < (1L << 31), "grid_sample3d_bwd_input: more than 2^31 voxels or cells");
  hipStream_t s = (hipStream_t)stream;
  const long ncell = (long)(B / group) * Di * Hi * Wi;
  const hipError_t me = hipMemsetAsync(w.cnt, 0, w.nkey * sizeof(int), s);
  FV_REQUIRE(me == hipSuccess, "grid_sample3d_bwd_input: hipMemsetAsync: %s", hipGetErrorString(me));
  hipLaunchKernelGGL(gs_bucket_count, dim3(fv_cdiv(w.nvox, 256)), dim3(256), 0, s, grid, w.nvox, (long)Do * Ho * Wo, Di,
                     Hi, Wi, group, w.cnt, w.keyrank);
  hipLaunchKernelGGL(gs_scan_blocks, dim3((unsigned)w.nblk), dim3(256), 0, s, w.cnt, w.nkey, w.bsum);
  hipLaunchKernelGGL(gs_scan_totals, dim3(1), dim3(256), 0, s, w.bsum, (int)w.nblk, w.lst);
  hipLaunchKernelGGL(gs_bucket_fill, dim3(fv_cdiv(w.nvox, 256)), dim3(256), 0, s, grid, w.keyrank, w.cnt, w.bsum,
                     w.nvox, Di, Hi, Wi, w.rec);
  hipLaunchKernelGGL(gs_bucket_sort, dim3(fv_cdiv(w.nkey - 1, 256)), dim3(256), 0, s, w.rec, w.cnt, w.bsum, w.nkey,
                     w.lst, w.midk, w.bigk);
  hipLaunchKernelGGL(gs_bucket_sort_coop, dim3(GS_COOP_BLOCKS), dim3(256), 0, s, grid, w.keyrank, w.rec, w.cnt, w.bsum,
                     w.lst, w.midk, w.bigk, w.nvox, Di, Hi, Wi);
#define GS_GATHER(T, V)                                                                                          \
  hipLaunchKernelGGL((gs_gather_input<T, V>), dim3(fv_cdiv(ncell * (C / V), 256)), dim3(256), 0, s, w.rec, w.cnt, \
                     w.bsum, (const T*)gout, ncell, Di, Hi, Wi, C, (T*)gin)
  // C = 32 (the warp volume): one lane per cell, its record read once (r4: 4 lanes of 8
  // channels each re-read every record)
  // (88.0 -> 73.6 us at the fbench shape, tools/r4ao.sh)
  if (dtype == FV_BF16) {
    if (C == 32) GS_GATHER(bf16, 32); else if (C % 8 == 0) GS_GATHER(bf16, 8); else GS_GATHER(bf16, 1);
  } else {
    if (C == 32) GS_GATHER(float, 32); else if (C % 8 == 0) GS_GATHER(float, 8); else GS_GATHER(float, 1);
  }
#undef GS_GATHER
  return fv_check_launch("grid_sample3d_bwd_input");
}

int fv_f32_to(int dtype, const float* a, void* b, long n, void* stream) {
  FV_REQUIRE(a && b && n >= 0, "f32_to: bad argument");
  if (n == 0) return FV_OK;
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16) hipLaunchKernelGGL(f32_to_kernel<bf16>, dim3(fv_cdiv(n, 256)), dim3(256), 0, s, a, (bf16*)b, n);
  else hipLaunchKernelGGL(f32_to_kernel<float>, dim3(fv_cdiv(n, 256)), dim3(256), 0, s, a, (float*)b, n);
  return fv_check_launch("f32_to");
}

int fv_occlusion_fwd(int dtype, const void* x, const float* occ, long P, int C, void* y, void* stream) {
  FV_REQUIRE(x && occ && y && P > 0 && C > 0, "occlusion: bad argument");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(occlusion_fwd<bf16>, dim3(fv_cdiv(P, 4)), dim3(256), 0, s, (const bf16*)x, occ, (bf16*)y, P, C);
  else
    hipLaunchKernelGGL(occlusion_fwd<float>, dim3(fv_cdiv(P, 4)), dim3(256), 0, s, (const float*)x, occ, (float*)y, P, C);
  return fv_check_launch("occlusion_fwd");
}

int fv_occlusion_bwd(int dtype, const void* g, const void* x, const float* occ, long P, int C, void* dx, float* docc,
                     void* stream) {
  FV_REQUIRE(g && x && occ && P > 0 && C > 0, "occlusion_bwd: bad argument");
  hipStream_t s = (hipStream_t)stream;
  if (dtype == FV_BF16)
    hipLaunchKernelGGL(occlusion_bwd<bf16>, dim3(fv_cdiv(P, 4)), dim3(256), 0, s, (const bf16*)g, (const bf16*)x, occ,
                       (bf16*)dx, docc, P, C);
  else
    hipLaunchKernelGGL(occlusion_bwd<float>, dim3(fv_cdiv(P, 4)), dim3(256), 0, s, (const float*)g, (const float*)x,
                       occ, (float*)dx, docc, P, C);
  return fv_check_launch("occlusion_bwd");
}

int fv_sparse_motion_fwd(const float* kp_s, const float* kp_d, const float* J, int N, int K, int D, int H, int W,
                         float* out, void* stream) {
  FV_REQUIRE(kp_s && kp_d && J && out && N > 0 && K > 0 && D > 1 && H > 1 && W > 1, "sparse_motion: bad argument");
  const long n = (long)N * (K + 1) * D * H * W;
  hipLaunchKernelGGL(sparse_motion_fwd, dim3(fv_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, kp_s, kp_d, J, out,
                     N, K, D, H, W);
  return fv_check_launch("sparse_motion_fwd");
}

/* sums [N][K][12]: (sum_v g, sum_v g c^T) of each keypoint's motion gradient */
int fv_sparse_motion_bwd(const float* g, const float* kp_d, int N, int K, int D, int H, int W, float* sums,
                         void* stream) {
  FV_REQUIRE(g && kp_d && sums && N > 0 && K > 0, "sparse_motion_bwd: bad argument");
  hipLaunchKernelGGL(sparse_motion_bwd, dim3(N * K), dim3(256), 0, (hipStream_t)stream, g, kp_d, sums, N, K, D, H, W);
  return fv_check_launch("sparse_motion_bwd");
}

int fv_heatmap_fwd(const float* kp_s, const float* kp_d, int N, int K, int D, int H, int W, float var, float* out,
                   void* stream) {
  FV_REQUIRE(kp_s && kp_d && out && N > 0 && K > 0 && D > 1 && H > 1 && W > 1, "heatmap: bad argument");
  const long n = (long)N * (K + 1) * D * H * W;
  hipLaunchKernelGGL(heatmap_fwd, dim3(fv_cdiv(n, 256)), dim3(256), 0, (hipStream_t)stream, kp_s, kp_d, out, N, K, D,
                     H, W, var);
  return fv_check_launch("heatmap_fwd");
}

int fv_heatmap_bwd(const float* g, const float* kp_s, const float* kp_d, int N, int K, int D, int H, int W, float var,
                   float* dkp_s, float* dkp_d, void* stream) {
  FV_REQUIRE(g && kp_s && kp_d && dkp_s && dkp_d && N > 0 && K > 0, "heatmap_bwd: bad argument");
  hipLaunchKernelGGL(heatmap_bwd, dim3(N * K), dim3(256), 0, (hipStream_t)stream, g, kp_s, kp_d, dkp_s, dkp_d, N, K,
                     D, H, W, var);
  return fv_check_launch("heatmap_bwd");
}

int fv_motion_mask_fwd(const float* logits, const float* sm, int N, int K1, long V, float* prob, float* def,
                       void* stream) {
  FV_REQUIRE(logits && sm && def && N > 0 && K1 > 0 && V > 0, "motion_mask: bad argument");
  hipLaunchKernelGGL(motion_mask_fwd, dim3(fv_cdiv((long)N * V, 256)), dim3(256), 0, (hipStream_t)stream, logits, sm,
                     prob, def, N, K1, V);
  return fv_check_launch("motion_mask_fwd");
}

int fv_motion_mask_bwd(const float* prob, const float* sm, const float* gdef, const float* gprob, int N, int K1,
                       long V, float* dlogits, float* dsm, void* stream) {
  FV_REQUIRE(prob && sm && gdef && N > 0 && K1 > 0 && V > 0, "motion_mask_bwd: bad argument");
  hipLaunchKernelGGL(motion_mask_bwd, dim3(fv_cdiv((long)N * V, 256)), dim3(256), 0, (hipStream_t)stream, prob, sm,
                     gdef, gprob, dlogits, dsm, N, K1, V);
  return fv_check_launch("motion_mask_bwd");
}

}  // extern "C"
