// On-the-fly ("alternate") correlation of the alt_cuda_corr plugin and the NHWC
// average pool of AlternateCorrBlock's feature pyramid (gfx950).
#include "common.hpp"

namespace raft {
namespace {

using h4 = __attribute__((ext_vector_type(4))) _Float16;
using h8 = __attribute__((ext_vector_type(8))) _Float16;

// ============================================================================
// K3: on-the-fly correlation (alt_cuda_corr forward, correlation_kernel.cu:18-119)
//
// One wave per (query pixel, coordinate set).  fmap1[p] is held in registers,
// 4 channels per lane per 256-channel slab.  The (2r+2)^2 integer taps
// around floor(coords) - r are visited 64 at a time: every lane reads the
// tap's fmap2 row slice (one coalesced 1 KiB read per tap per slab) and keeps
// a private partial dot product per tap; per batch of 8 taps a transposing
// butterfly (7 shuffles) and 3 lane-group butterflies leave lane j holding tap
// j's full sum.  The tap loads are branch-free buffer loads (out-of-map taps
// read zeros), issued a batch ahead of the products.
// Tap sums go to LDS and the bilinear weights of frac(coords) scatter them
// into the (2r+1)^2 bins exactly as the reference (bins gathered per lane).
// ============================================================================
struct AltArgs {
  const float* f1;
  const float* f2;
  const float* coords;
  int coords_layout;  // 0 = [B][N][H1][W1][2] (reference) / NHWC rows, 1 = NCHW [B][2][H1][W1]
  float coord_div;
  float* out;
  int out_layout;  // 0 = [B][N][RD^2][H1][W1] (reference), 1 = NHWC rows out_ld
  int out_ld;
  int B, H1, W1, H2, W2, C, N, r;
  float scale_div;
  float* flow;
  int flow_ld;
  int* range_flag;  // f16x3 range guard (raft_hip.h), or null
  int prec;         // RAFT_PREC_FP32: exact fp32 (VALU kernels); otherwise the f16x3 box GEMM where it applies
};

// One tap's fmap2 row slice for this lane's channel quads, read through a raw
// buffer over the batch's fmap2.  An out-of-map (or beyond-C) read passes an
// out-of-range offset and returns zeros without a memory access, so every
// tap's load is issued unconditionally — no exec-masked branch per tap, and
// a batch of taps goes out back to back instead of one L2 round trip per tap.
template <int NV>
__device__ __forceinline__ void tap_load(f32x4 (&d)[NV], __amdgpu_buffer_rsrc_t rs, bool in, int row_off, int lane,
                                         int C) {
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = k * 256 + lane * 4;
    const unsigned off = (in && c < C) ? (unsigned)(row_off + c) * 4u : 0x80000000u;
    d[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
  }
}

template <int NV>
__device__ __forceinline__ float tap_dot(const f32x4 (&f1)[NV], const f32x4 (&d)[NV]) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) s += f1[k][0] * d[k][0] + f1[k][1] * d[k][1] + f1[k][2] * d[k][2] + f1[k][3] * d[k][3];
  return s;
}

// Reduce v[0..N-1] (one partial per tap, per lane) so that lane l ends with the
// sum over its N-lane group (lanes sharing l / N) of v[l % N]: log2(N) halving
// exchanges, N - 1 shuffles.
template <int N>
__device__ __forceinline__ float transpose_reduce(float (&v)[N], int lane) {
#pragma unroll
  for (int half = N / 2; half >= 1; half >>= 1) {
    const bool hi = (lane & half) != 0;
#pragma unroll
    for (int i = 0; i < half; ++i) {
      const float keep = hi ? v[i + half] : v[i];
      const float send = hi ? v[i] : v[i + half];
      v[i] = keep + __shfl_xor(send, half);
    }
  }
  return v[0];
}

// waves per SIMD the forward kernel is compiled for at C <= 256 (8 / NV above; register budget: its tap
// group's loads all in flight vs more waves); dev builds may override it
#ifndef ALT_WAVES
#define ALT_WAVES 8
#endif
#ifndef ALT_PF  // 1: the next batch's loads go out before this batch's products
#define ALT_PF 1
#endif
#ifndef ALT_TB  // taps per load batch
#define ALT_TB 2
#endif
// One query pixel gid = (b*N + n)*P1 + p by one wave (ts: the wave's 128-float
// LDS row of tap sums).
template <int NV>
__device__ __forceinline__ void alt_pixel(const AltArgs& a, long gid, bool valid, int lane, float* ts) {
  const int P1 = a.H1 * a.W1;
  const long bn = valid ? gid / P1 : 0;
  const int p = valid ? (int)(gid - bn * P1) : 0;
  const int b = (int)(bn / a.N);
  const int rd = 2 * a.r + 1, wd = 2 * a.r + 2, ntaps = wd * wd;

  float x = 0.f, y = 0.f;
  if (valid) {
    if (a.coords_layout == 0) {
      x = a.coords[2 * gid];
      y = a.coords[2 * gid + 1];
    } else {
      x = a.coords[((long)b * 2) * P1 + p];
      y = a.coords[((long)b * 2 + 1) * P1 + p];
    }
    x = x / a.coord_div;
    y = y / a.coord_div;
  }
  const float fx = floorf(x), fy = floorf(y);
  const float dx = x - fx, dy = y - fy;
  const int x0 = (int)fx - a.r, y0 = (int)fy - a.r;

  f32x4 f1[NV];
  const float* f1row = a.f1 + ((long)b * P1 + p) * a.C;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = k * 256 + lane * 4;
    f1[k] = (valid && c < a.C) ? *reinterpret_cast<const f32x4*>(f1row + c) : f32x4{0.f, 0.f, 0.f, 0.f};
  }
  const float* f2b = a.f2 + (long)b * a.H2 * a.W2 * a.C;
  // < 2 GiB per batch item (host-checked)
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(f2b), (short)0, (int)((long)a.H2 * a.W2 * a.C * 4), 0x00020000);
  // the window origin is the wave's (one pixel per wave): scalar tap geometry
  const int sx0 = __builtin_amdgcn_readfirstlane(x0), sy0 = __builtin_amdgcn_readfirstlane(y0);
  // taps in batches of TB: batch k + 1's loads are issued before batch k's
  // products, so each wave keeps 2 x TB tap rows in flight
  constexpr int TB = ALT_TB;
  auto tap_in = [&](int t, int& row_off) {
    const int iy = t / wd, ix = t - iy * wd;
    const int h2 = sy0 + iy, w2 = sx0 + ix;
    row_off = (h2 * a.W2 + w2) * a.C;
    return valid && t < ntaps && (unsigned)h2 < (unsigned)a.H2 && (unsigned)w2 < (unsigned)a.W2;
  };
  for (int g = 0; g < ntaps; g += 64) {
    f32x4 buf[ALT_PF ? 2 : 1][TB][NV];
#pragma unroll
    for (int j = 0; j < TB; ++j) {
      int ro;
      const bool in = tap_in(g + j, ro);
      tap_load<NV>(buf[0][j], rs, in, ro, lane, a.C);
    }
#pragma unroll
    for (int jb = 0; jb < 64; jb += TB) {
      if (g + jb >= ntaps) break;  // wave-uniform
      const int cur = ALT_PF ? (jb / TB) & 1 : 0;
      if (!ALT_PF && jb > 0) {
#pragma unroll
        for (int j = 0; j < TB; ++j) {
          int ro;
          const bool in = tap_in(g + jb + j, ro);
          tap_load<NV>(buf[0][j], rs, in, ro, lane, a.C);
        }
      }
      if (ALT_PF && jb + TB < 64) {
#pragma unroll
        for (int j = 0; j < TB; ++j) {
          int ro;
          const bool in = tap_in(g + jb + TB + j, ro);
          tap_load<NV>(buf[ALT_PF ? cur ^ 1 : 0][j], rs, in, ro, lane, a.C);
        }
      }
      __builtin_amdgcn_sched_barrier(0);
      float v[TB];
#pragma unroll
      for (int j = 0; j < TB; ++j) v[j] = tap_dot<NV>(f1, buf[cur][j]);
      // lane l ends with the full sum of tap jb + (l % TB): a transposing
      // butterfly over the batch, then a plain one over the lane groups
      float tot = transpose_reduce<TB>(v, lane);
#pragma unroll
      for (int m = TB; m < 64; m <<= 1) tot += __shfl_xor(tot, m);
      if (lane < TB && g + jb + lane < ntaps) ts[g + jb + lane] = tot;
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (!valid) return;
  for (int o = lane; o < rd * rd; o += 64) {
    const int ox = o / rd, oy = o - ox * rd;  // channel = oy + rd*ox
    const float s00 = ts[oy * wd + ox], s01 = ts[oy * wd + ox + 1];
    const float s10 = ts[(oy + 1) * wd + ox], s11 = ts[(oy + 1) * wd + ox + 1];
    float val = s00 * ((1.f - dy) * (1.f - dx));
    val += s01 * ((1.f - dy) * dx);
    val += s10 * (dy * (1.f - dx));
    val += s11 * (dy * dx);
    val = val / a.scale_div;
    if (a.range_flag && fabsf(val) > RAFT_RANGE_LIMIT) *a.range_flag = 1;
    if (a.out_layout == 0)
      a.out[(bn * (rd * rd) + o) * P1 + p] = val;
    else
      a.out[((long)b * P1 + p) * a.out_ld + o] = val;
  }
  if (a.flow && lane < 2) {
    const float gx = lane == 0 ? (float)(p % a.W1) : (float)(p / a.W1);
    a.flow[((long)b * P1 + p) * a.flow_ld + lane] = (lane == 0 ? x : y) * a.coord_div - gx;
  }
}


template <int NV>
__global__ __launch_bounds__(256, NV == 1 ? ALT_WAVES : 8 / NV) void alt_corr_kernel(AltArgs a) {
  __shared__ float tapsum[4][128];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const long gid = (long)blockIdx.x * 4 + wv;  // ((b*N + n)*P1 + p)
  alt_pixel<NV>(a, gid, gid < (long)a.B * a.N * a.H1 * a.W1, lane, tapsum[wv]);
}

// ============================================================================
// K3t: tiled on-the-fly correlation (the same forward, correlation_kernel.cu:18-119).
//
// One 256-thread work-group per 8x8 tile of query pixels and coordinate set.
// Neighbouring pixels' (2r+2)^2 windows overlap, so the union of the tile's
// windows (its bounding box, <= ATB x ATB fmap2 pixels) is staged in LDS one
// ACC-channel chunk at a time (ACC = 8, ATB = 28: 37 KB of LDS, 4 waves/SIMD;
// 16 channels was 5 % slower at 3 waves/SIMD; a 24-pixel box sent 30 % more
// tiles of a divergent field to the per-pixel path) and every (pixel, tap) dot product reads it from
// there: fmap2 crosses L2 once per tile instead of once per pixel and tap
// (the per-pixel kernel above moves 100 KiB per pixel and level).  Thread
// (g, q) = (wave, lane) accumulates taps g, g + 4, ... of tile pixel q; its
// fmap1 chunk sits in registers.  A tile whose box does not fit (large flow
// divergence, non-finite coords) is finished per pixel by its waves
// (alt_pixel, the per-pixel kernel's body).  Bilinear binning and the output layouts are those of
// alt_corr_kernel.
// ============================================================================
constexpr int AT = 8;     // tile side (query pixels)
#ifndef ALT_ACC  // (dev builds may override the chunk and box sizes)
#define ALT_ACC 8
#endif
#ifndef ALT_ATB
#define ALT_ATB 28
#endif
constexpr int ACC = ALT_ACC;  // channels per staged chunk
constexpr int ATB = ALT_ATB;  // max bounding-box side (fmap2 pixels)

// bilinear binning of one pixel's tap sums ts[(2r+2)^2] into output channel o
__device__ __forceinline__ void alt_bin_store(const AltArgs& a, long bn, int p, float x, float y, const float* ts,
                                              int o) {
  const int P1 = a.H1 * a.W1;
  const int b = (int)(bn / a.N);
  const int rd = 2 * a.r + 1, wd = 2 * a.r + 2;
  const float fx = floorf(x), fy = floorf(y);
  const float dx = x - fx, dy = y - fy;
  const int ox = o / rd, oy = o - ox * rd;  // channel = oy + rd*ox
  const float s00 = ts[oy * wd + ox], s01 = ts[oy * wd + ox + 1];
  const float s10 = ts[(oy + 1) * wd + ox], s11 = ts[(oy + 1) * wd + ox + 1];
  float val = s00 * ((1.f - dy) * (1.f - dx));
  val += s01 * ((1.f - dy) * dx);
  val += s10 * (dy * (1.f - dx));
  val += s11 * (dy * dx);
  val = val / a.scale_div;
  if (a.range_flag && fabsf(val) > RAFT_RANGE_LIMIT) *a.range_flag = 1;
  if (a.out_layout == 0)
    a.out[(bn * (rd * rd) + o) * P1 + p] = val;
  else
    a.out[((long)b * P1 + p) * a.out_ld + o] = val;
}

template <int R>
__global__ __launch_bounds__(256) void alt_corr_tile_kernel(AltArgs a) {
  constexpr int WD = 2 * R + 2, NT = WD * WD, RD = 2 * R + 1;
  constexpr int TPT = (NT + 3) / 4;  // taps per thread
  constexpr int SROW = ACC + 4;      // staged floats per box pixel (16-B pad against bank conflicts)
  __shared__ __attribute__((aligned(16))) float st[ATB * ATB * SROW > AT * AT * (NT + 1) ? ATB * ATB * SROW
                                                                                       : AT * AT * (NT + 1)];
  const int lane = threadIdx.x & 63;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int P1 = a.H1 * a.W1;
  const int tiles_x = (a.W1 + AT - 1) / AT, tiles_y = (a.H1 + AT - 1) / AT;
  const int per = tiles_x * tiles_y;
  const long bn = blockIdx.x / per;
  const int tr = (int)(blockIdx.x - bn * per);
  const int b = (int)(bn / a.N);
  const int qy = (tr / tiles_x) * AT + (lane >> 3), qx = (tr % tiles_x) * AT + (lane & 7);
  const bool valid = qy < a.H1 && qx < a.W1;
  const int p = valid ? qy * a.W1 + qx : 0;
  const long gid = bn * P1 + p;

  float x = 0.f, y = 0.f;
  if (valid) {
    if (a.coords_layout == 0) {
      x = a.coords[2 * gid];
      y = a.coords[2 * gid + 1];
    } else {
      x = a.coords[((long)b * 2) * P1 + p];
      y = a.coords[((long)b * 2 + 1) * P1 + p];
    }
    x = x / a.coord_div;
    y = y / a.coord_div;
  }
  const bool fin = isfinite(x) && isfinite(y) && fabsf(x) < 1e8f && fabsf(y) < 1e8f;
  const int x0 = fin ? (int)floorf(x) - R : 0, y0 = fin ? (int)floorf(y) - R : 0;
  // the tile's window box (every wave computes the same one)
  int mnx = valid ? x0 : (1 << 30), mny = valid ? y0 : (1 << 30);
  int mxx = valid ? x0 : -(1 << 30), mxy = valid ? y0 : -(1 << 30);
  int bad = valid && !fin;
#pragma unroll
  for (int m = 1; m < 64; m <<= 1) {
    mnx = min(mnx, __shfl_xor(mnx, m));
    mny = min(mny, __shfl_xor(mny, m));
    mxx = max(mxx, __shfl_xor(mxx, m));
    mxy = max(mxy, __shfl_xor(mxy, m));
    bad |= __shfl_xor(bad, m);
  }
  const int bx0 = __builtin_amdgcn_readfirstlane(mnx), by0 = __builtin_amdgcn_readfirstlane(mny);
  const int bw = __builtin_amdgcn_readfirstlane(mxx) - bx0 + WD, bh = __builtin_amdgcn_readfirstlane(mxy) - by0 + WD;
  const bool fits = !__builtin_amdgcn_readfirstlane(bad) && bw <= ATB && bh <= ATB;

  if (!fits) {
    // wave g finishes pixels 16g .. 16g + 15 of the tile one at a time (per-pixel path)
    for (int i = 0; i < 16; ++i) {
      const int q = 16 * g + i;
      const int pq = __shfl(p, q), vq = __shfl((int)valid, q);
      alt_pixel<1>(a, bn * P1 + pq, vq != 0, lane, st + g * 128);
    }
    return;
  }

  // box-relative window origin of this thread's pixel
  const int ox0 = valid ? x0 - bx0 : 0, oy0 = valid ? y0 - by0 : 0;
  const float* f2b = a.f2 + (long)b * a.H2 * a.W2 * a.C;
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
      const_cast<float*>(f2b), (short)0, (int)((long)a.H2 * a.W2 * a.C * 4), 0x00020000);
  const float* f1row = a.f1 + ((long)b * P1 + p) * a.C;
  float acc[TPT];
#pragma unroll
  for (int j = 0; j < TPT; ++j) acc[j] = 0.f;
  constexpr int PIECES = ATB * ATB * (ACC / 4);  // 16-B pieces of a full box chunk
  const int npieces = bw * bh * (ACC / 4);
  for (int c0 = 0; c0 < a.C; c0 += ACC) {
    // stage the box's chunk: piece i = (box pixel i / (ACC/4), quad i % (ACC/4)); zeros off the map
    f32x4 v[(PIECES + 255) / 256];
#pragma unroll
    for (int k = 0; k < (PIECES + 255) / 256; ++k) {
      const int i = threadIdx.x + 256 * k;
      const int bp = i / (ACC / 4), qd = i % (ACC / 4);
      const int yy = bp / bw, xx = bp - (bp / bw) * bw;
      const int h2 = by0 + yy, w2 = bx0 + xx;
      const bool in = i < npieces && (unsigned)h2 < (unsigned)a.H2 && (unsigned)w2 < (unsigned)a.W2;
      const unsigned off = in ? (unsigned)((h2 * a.W2 + w2) * a.C + c0 + 4 * qd) * 4u : 0x80000000u;
      v[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
    f32x4 f1c[ACC / 4];
#pragma unroll
    for (int k = 0; k < ACC / 4; ++k) f1c[k] = *reinterpret_cast<const f32x4*>(f1row + c0 + 4 * k);
    __syncthreads();  // the previous chunk's reads are done
#pragma unroll
    for (int k = 0; k < (PIECES + 255) / 256; ++k) {
      const int i = threadIdx.x + 256 * k;
      if (i < npieces) {
        const int bp = i / (ACC / 4), qd = i % (ACC / 4);
        const int yy = bp / bw, xx = bp - (bp / bw) * bw;
        *reinterpret_cast<f32x4*>(&st[(yy * ATB + xx) * SROW + 4 * qd]) = v[k];
      }
    }
    __syncthreads();
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
      const int t = g + 4 * j;
      if (t < NT) {
        const int iy = t / WD, ix = t - (t / WD) * WD;
        const float* sp = &st[((oy0 + iy) * ATB + ox0 + ix) * SROW];
        float s = 0.f;
#pragma unroll
        for (int k = 0; k < ACC / 4; ++k) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(sp + 4 * k);
          s += f1c[k][0] * u[0] + f1c[k][1] * u[1] + f1c[k][2] * u[2] + f1c[k][3] * u[3];
        }
        acc[j] += s;
      }
    }
  }
  __syncthreads();
  // tap sums of the tile's pixels: ts[q][t] (reusing the staging area)
  float* ts = st + lane * (NT + 1);
#pragma unroll
  for (int j = 0; j < TPT; ++j) {
    const int t = g + 4 * j;
    if (t < NT) ts[t] = acc[j];
  }
  __syncthreads();
  if (a.out_layout == 1) {
    // NHWC rows: wave g writes pixels g, g + 4, ... with lanes along the row
    // (a pixel-per-lane store would scatter 4-B writes 324 floats apart)
    for (int q = g; q < AT * AT; q += 4) {
      const float xq = __shfl(x, q), yq = __shfl(y, q);
      const int pq = __shfl(p, q), vq = __shfl((int)valid, q);
      if (!vq) continue;
      for (int o = lane; o < RD * RD; o += 64) alt_bin_store(a, bn, pq, xq, yq, st + q * (NT + 1), o);
    }
    if (!valid) return;
  } else {
    if (!valid) return;
    for (int o = g; o < RD * RD; o += 4) alt_bin_store(a, bn, p, x, y, ts, o);
  }
  if (a.flow && g == 0) {
    a.flow[((long)b * P1 + p) * a.flow_ld + 0] = x * a.coord_div - (float)(p % a.W1);
    a.flow[((long)b * P1 + p) * a.flow_ld + 1] = y * a.coord_div - (float)(p / a.W1);
  }
}

// ============================================================================
// K3m: the tile kernel's tap sums on MFMA (RAFT: C = 256, r = 4).
//
// The tap sums of an 8x8 query tile are dot products of its 64 fmap1 rows with
// the fmap2 pixels of the tile's window box: a GEMM S = F1 * F2box^T (M = 64
// queries, N = box pixels, K = C) of which each query keeps its (2r+2)^2 window
// entries.  The VALU tile kernel reads LDS once per (query, tap, 8 channels);
// here the box (up to 96 x 96 fmap2 pixels, where the VALU kernel stops at 28 x 28)
// is consumed in bands of whole box rows (96 / box width of them, N padded to 96) on v_mfma_f32_32x32x16_f16 in the fp32-accurate split (hi*hi + lo*hi +
// hi*lo, the corr_build arithmetic), and the band's 64 x 64 product goes through
// LDS where every query picks the taps of its window that lie in the band.
//   LDS: F1 tile, all K, split (64 x C/32 x 128 B = 64 KB) | band rows of F2
//   (96 px x C/32 x 128 B, reused for the band's S) -> 160 KB, one work-group
//   per CU; 8 waves load, waves 0-5 own one 32x32 S subtile each, all 8 pick taps.
// The next band's fmap2 loads are issued before the current band's MFMAs.
// ============================================================================
#ifndef ALT_MFMA16
#define ALT_MFMA16 1  // the box GEMM on 16x16 blocks: 1 = 8 waves, 2 = 4 waves of 32 rows (0: 6 waves of 32x32 blocks)
#endif
constexpr int AM_KS = 8;                 // 32-channel K-steps (C <= 256)
constexpr int AM_ROW = 128;              // bytes per (row, K-step): 32 hi | 32 lo halves, 16-B chunks
                                         // XOR-swizzled by row & 7 (conflict-free fragment reads)
constexpr int AM_NB = 96;                // band pixels (>= 3 box rows of ATB)
constexpr int AM_SLD = AM_NB + 4;        // S row stride (floats)
constexpr int AM_PER = AM_NB * AM_KS * 32 / 4 / 512;  // 16-B loads per thread per band (C = 256): 12

// byte offset of logical 16-B chunk c of LDS row `row`
__device__ __forceinline__ int am_chunk(int row, int c) { return ((c ^ (row & 7)) << 4); }

// 4 floats (channels 4*quad .. +3 of a K-step) -> f16 hi in chunk quad/2, lo = f16(x - hi) in
// chunk 4 + quad/2 (the corr_build split, unscaled lo)
__device__ __forceinline__ void am_split_store(char* base, int row, int quad, f32x4 v) {
  h4 hi, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 h = (_Float16)v[e];
    hi[e] = h;
    lo[e] = (_Float16)(v[e] - (float)h);
  }
  char* r = base + row * AM_ROW + (quad & 1) * 8;
  *reinterpret_cast<h4*>(r + am_chunk(row, quad >> 1)) = hi;
  *reinterpret_cast<h4*>(r + am_chunk(row, 4 + (quad >> 1))) = lo;
}

// the per-level operands of one launch over all levels (raft_alt_corr_lookup_levels)
constexpr int AM_MAXL = 6;
struct AltLevels {
  const float* f2[AM_MAXL];
  float* out[AM_MAXL];
  int H2[AM_MAXL], W2[AM_MAXL];
  float div[AM_MAXL];
  int n;
};

// the per-pixel path of a tile whose box does not fit, out of line (rare: keeps its registers out
// of the MFMA tile kernel's main path)
__device__ __noinline__ void alt_pixel_ni(const AltArgs& a, long gid, bool valid, int lane, float* ts) {
  alt_pixel<1>(a, gid, valid, lane, ts);
}

#ifdef ALT_STAMPS  // dev-only phase timing (tools/alt_stamps.py with a -DALT_STAMPS variant)
__device__ unsigned long long g_altstamp[24 * 8 * 4096];
__device__ __forceinline__ unsigned long long alt_clock() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
// phase k gets the cycles since the previous stamp
#define ALT_ST(k)                       \
  do {                                  \
    const unsigned long long n_ = alt_clock(); \
    alt_t[k] += n_ - alt_prev;          \
    alt_prev = n_;                      \
  } while (0)
#else
#define ALT_ST(k)
#endif

template <int R>
__global__ __launch_bounds__(512) void alt_corr_mfma_kernel(AltArgs a0, AltLevels lvs) {
#ifdef ALT_STAMPS
  unsigned long long alt_t[16] = {}, alt_prev = alt_clock();
  const unsigned long long alt_start = alt_prev;
  int alt_bands = 0;
#endif
  constexpr int WD = 2 * R + 2, NT = WD * WD, RD = 2 * R + 1;
  constexpr int TPT = (NT + 7) / 8;  // taps per thread (8 waves)
  constexpr int ABYTES = AT * AT * AM_KS * AM_ROW, BBYTES = AM_NB * AM_KS * AM_ROW;
  static_assert(AM_NB * AM_SLD * 4 <= BBYTES && AT * AT * (NT + 1) * 4 + AT * AT * 16 <= BBYTES,
                "S and ts (+ the query table) fit the band region");
  __shared__ __attribute__((aligned(16))) char smem[ABYTES + BBYTES];
  char* const As = smem;                // the F1 tile: resident over all levels
  char* const Bs = smem + ABYTES;       // band rows, then the band's S, then the tap sums
  float* const S = reinterpret_cast<float*>(Bs);
  const int lane = threadIdx.x & 63;
  const int g = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // wave 0..7
  const int tid = threadIdx.x;
  const int P1 = a0.H1 * a0.W1;
  const int tiles_x = (a0.W1 + AT - 1) / AT, tiles_y = (a0.H1 + AT - 1) / AT;
  const int per = tiles_x * tiles_y;
  const long bn = blockIdx.x / per;
  const int tr = (int)(blockIdx.x - bn * per);
  const int b = (int)(bn / a0.N);
  // every wave holds the tile's 64 queries, one per lane (the box is computed per wave)
  const int qy = (tr / tiles_x) * AT + (lane >> 3), qx = (tr % tiles_x) * AT + (lane & 7);
  const bool valid = qy < a0.H1 && qx < a0.W1;
  const int p = valid ? qy * a0.W1 + qx : 0;
  const long gid = bn * P1 + p;
  float xr = 0.f, yr = 0.f;  // level-0 coordinates
  if (valid) {
    if (a0.coords_layout == 0) {
      xr = a0.coords[2 * gid];
      yr = a0.coords[2 * gid + 1];
    } else {
      xr = a0.coords[((long)b * 2) * P1 + p];
      yr = a0.coords[((long)b * 2 + 1) * P1 + p];
    }
  }
  const int ks = a0.C / 32;  // K-steps (host-checked: C % 32 == 0, C <= 256)
  // ---- F1 tile -> LDS (split), all K, once for every level: thread = (query q, 16-B quad qd)
  {
    constexpr int AQ = AT * AT * AM_KS * 8 / 512;
    const float* f1b = a0.f1 + (long)b * P1 * a0.C;
    f32x4 av[AQ];
#pragma unroll
    for (int k = 0; k < AQ; ++k) {
      const int i = tid + 512 * k, q = i >> 6, qd = i & 63;
      const int qyy = (tr / tiles_x) * AT + (q >> 3), qxx = (tr % tiles_x) * AT + (q & 7);
      const bool v = qyy < a0.H1 && qxx < a0.W1 && 4 * qd < a0.C;
      av[k] = v ? *reinterpret_cast<const f32x4*>(f1b + ((long)qyy * a0.W1 + qxx) * a0.C + 4 * qd)
                : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < AQ; ++k) {
      const int i = tid + 512 * k, q = i >> 6, qd = i & 63, s = qd >> 3;
      if (s < ks) am_split_store(As, s * (AT * AT) + q, qd & 7, av[k]);
    }
  }
  ALT_ST(0);  // F1 tile
#if !ALT_MFMA16
  const int mi = g & 1, ni = g >> 1;  // S subtile of MFMA waves 0-5
  const int m = lane & 31, h = lane >> 5;
#endif
  // ---- per-level window box (wave-uniform) and the band loads, set up one level ahead ------
  struct Lvl {
    float x, y;       // this lane's query at the level
    int x0, y0;       // its window origin
    int bx0, by0, bw, bh, br;  // the tile's box and box rows per band
    bool fits;
  };
  auto setup = [&](int l, Lvl& v) {
    const float div = lvs.div[l];
    v.x = valid ? xr / div : 0.f;
    v.y = valid ? yr / div : 0.f;
    const bool fin = isfinite(v.x) && isfinite(v.y) && fabsf(v.x) < 1e8f && fabsf(v.y) < 1e8f;
    v.x0 = fin ? (int)floorf(v.x) - R : 0;
    v.y0 = fin ? (int)floorf(v.y) - R : 0;
    int mnx = valid ? v.x0 : (1 << 30), mny = valid ? v.y0 : (1 << 30);
    int mxx = valid ? v.x0 : -(1 << 30), mxy = valid ? v.y0 : -(1 << 30);
    int bad = valid && !fin;
#pragma unroll
    for (int k = 1; k < 64; k <<= 1) {
      mnx = min(mnx, __shfl_xor(mnx, k));
      mny = min(mny, __shfl_xor(mny, k));
      mxx = max(mxx, __shfl_xor(mxx, k));
      mxy = max(mxy, __shfl_xor(mxy, k));
      bad |= __shfl_xor(bad, k);
    }
    v.bx0 = __builtin_amdgcn_readfirstlane(mnx);
    v.by0 = __builtin_amdgcn_readfirstlane(mny);
    v.bw = __builtin_amdgcn_readfirstlane(mxx) - v.bx0 + WD;
    v.bh = __builtin_amdgcn_readfirstlane(mxy) - v.by0 + WD;
    // any box up to AM_NB wide is consumed band by band (a tall box only costs more bands)
    v.fits = !__builtin_amdgcn_readfirstlane(bad) && v.bw <= AM_NB && v.bh <= AM_NB;
    v.br = v.fits ? AM_NB / v.bw : 1;  // box rows per band: as many whole rows as fit 96 pixels (>= 1)
  };
  // fmap2 band loads: thread = (band pixel j, quad) with j = g + 8k (wave-uniform), AM_PER per
  // thread; zeros off the map / band / channels
  f32x4 bv[AM_PER];
  auto load_band = [&](int l, const Lvl& v, int r0) {
    const int H2 = lvs.H2[l], W2 = lvs.W2[l];
    const float* f2b = lvs.f2[l] + (long)b * H2 * W2 * a0.C;
    const __amdgpu_buffer_rsrc_t rs =
        __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(f2b), (short)0, (int)((long)H2 * W2 * a0.C * 4), 0x00020000);
    const bool qin = 4 * lane < a0.C;
    int rr = 0, xx = g;  // (box row, column) of band pixel j = g + 8k (bw >= WD > 8: one wrap per step)
#pragma unroll
    for (int k = 0; k < AM_PER; ++k) {
      const int h2 = v.by0 + r0 + rr, w2 = v.bx0 + xx;
      const bool in = rr < v.br && r0 + rr < v.bh && (unsigned)h2 < (unsigned)H2 && (unsigned)w2 < (unsigned)W2;
      const unsigned off = (in && qin) ? (unsigned)((h2 * W2 + w2) * a0.C + 4 * lane) * 4u : 0x80000000u;
      bv[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      xx += 8;
      if (xx >= v.bw) {
        xx -= v.bw;
        ++rr;
      }
    }
  };
  auto store_band = [&]() {
#pragma unroll
    for (int k = 0; k < AM_PER; ++k) {
      const int j = g + 8 * k, s = lane >> 3;
#ifdef ALT_ABL_NOSPLIT  // dev ablation (wrong results): the band stored as loaded, one 16-B write per load
      if (s < ks) {
        const int row = s * AM_NB + j;
        *reinterpret_cast<f32x4*>(Bs + row * AM_ROW + am_chunk(row, lane & 7)) = bv[k];
      }
#else
      if (s < ks) am_split_store(Bs, s * AM_NB + j, lane & 7, bv[k]);
#endif
    }
  };
  Lvl cur;
  setup(0, cur);
  if (cur.fits) load_band(0, cur, 0);
  ALT_ST(1);  // level setup + first band issue
  for (int l = 0; l < lvs.n; ++l) {
    float* const out = lvs.out[l];
    const float cdiv = lvs.div[l];
    Lvl nxt = cur;
    if (!cur.fits) {
      // wave g finishes pixels 8g .. 8g + 7 of the tile one at a time (per-pixel path)
      AltArgs a = a0;
      a.f2 = lvs.f2[l];
      a.H2 = lvs.H2[l];
      a.W2 = lvs.W2[l];
      a.coord_div = cdiv;
      a.out = out;
      a.flow = l == 0 ? a0.flow : nullptr;
      float* ts = reinterpret_cast<float*>(Bs) + g * 128;
      for (int i = 0; i < 8; ++i) {
        const int q = 8 * g + i;
        const int pq = __shfl(p, q), vq = __shfl((int)valid, q);
        alt_pixel_ni(a, bn * P1 + pq, vq != 0, lane, ts);
      }
      __syncthreads();  // the band region is free for the next level
      if (l + 1 < lvs.n) {
        setup(l + 1, nxt);
        if (nxt.fits) load_band(l + 1, nxt, 0);
      }
      cur = nxt;
      continue;
    }
    // box-relative window origin of this lane's query; taps t = g + 8j
    const int ox0 = valid ? cur.x0 - cur.bx0 : 0, oy0 = valid ? cur.y0 - cur.by0 : 0;
    float tap[TPT];
#pragma unroll
    for (int j = 0; j < TPT; ++j) tap[j] = 0.f;
    for (int r0 = 0; r0 < cur.bh; r0 += cur.br) {
#ifdef ALT_STAMPS
      ++alt_bands;
#endif
      store_band();
      ALT_ST(2);  // band split + store (with the wait for its loads)
      __syncthreads();  // band r0 (and, first time round, the F1 tile) in LDS
      ALT_ST(3);
      if (r0 + cur.br < cur.bh) load_band(l, cur, r0 + cur.br);  // in flight under the MFMAs
      ALT_ST(4);
#if ALT_MFMA16
      // the band product on 16x16 blocks, every SIMD the same share.  ALT_MFMA16 == 1: all 8 waves,
      // wave g owns query rows 16 (g & 3) .. +15 x band pixels 48 (g >> 2) .. +47 (RB = 1 row block
      // of 3 column blocks); == 2: waves 0-3 (one per SIMD), wave g query rows 32 (g & 1) .. +31 x
      // band pixels 48 (g >> 1) .. +47 (RB = 2): the same MFMA cycles per SIMD from 37 % fewer LDS
      // fragment bytes (the 32x32 form ran on waves 0-5: SIMDs 0 and 1 carried two waves' MFMAs)
      constexpr int RB = ALT_MFMA16 == 2 ? 2 : 1;
      f32x4 c0[RB][3] = {}, c1[RB][3] = {}, c2[RB][3] = {};
      const int rb = RB == 2 ? (g & 1) : (g & 3), cg = RB == 2 ? (g >> 1) : (g >> 2);
      const int rl = lane & 15, kg = lane >> 4;
      if (RB == 1 || g < 4) {
        for (int s = 0; s < ks; ++s) {
          h8 xh[RB], xl[RB];
#pragma unroll
          for (int i = 0; i < RB; ++i) {
            const int ar = s * (AT * AT) + 16 * (RB * rb + i) + rl;
            const char* Ar = As + ar * AM_ROW;
            xh[i] = *reinterpret_cast<const h8*>(Ar + am_chunk(ar, kg));
            xl[i] = *reinterpret_cast<const h8*>(Ar + am_chunk(ar, 4 + kg));
          }
#pragma unroll
          for (int t = 0; t < 3; ++t) {
            const int brow = s * AM_NB + 48 * cg + 16 * t + rl;
            const char* Br = Bs + brow * AM_ROW;
            const h8 yh = *reinterpret_cast<const h8*>(Br + am_chunk(brow, kg));
            const h8 yl = *reinterpret_cast<const h8*>(Br + am_chunk(brow, 4 + kg));
#pragma unroll
            for (int i = 0; i < RB; ++i) {
              c0[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh[i], yh, c0[i][t], 0, 0, 0);
              c1[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xl[i], yh, c1[i][t], 0, 0, 0);
              c2[i][t] = __builtin_amdgcn_mfma_f32_16x16x32_f16(xh[i], yl, c2[i][t], 0, 0, 0);
            }
          }
        }
      }
      ALT_ST(5);  // MFMAs
      __syncthreads();  // every MFMA wave has read the band: its region takes S
      ALT_ST(6);
      // register r of block (i, t) holds S[query 16 (RB rb + i) + 4 kg + r][band pixel 48 cg + 16 t + rl]
      if (RB == 1 || g < 4) {
#pragma unroll
        for (int i = 0; i < RB; ++i)
#pragma unroll
          for (int t = 0; t < 3; ++t)
#pragma unroll
            for (int r = 0; r < 4; ++r)
              S[(16 * (RB * rb + i) + 4 * kg + r) * AM_SLD + 48 * cg + 16 * t + rl] =
                  c0[i][t][r] + c1[i][t][r] + c2[i][t][r];
      }
#else
      f32x16 acc = {}, acc2 = {}, acc3 = {};
      if (g < 6) {
        for (int s = 0; s < ks; ++s) {
          const int ar = s * (AT * AT) + 32 * mi + m, brow = s * AM_NB + 32 * ni + m;
          const char* Ar = As + ar * AM_ROW;
          const char* Br = Bs + brow * AM_ROW;
#pragma unroll
          for (int qq = 0; qq < 2; ++qq) {
            const int c = 2 * qq + h;  // the lane's 8 halves of this K-half: logical chunk c (hi), 4 + c (lo)
            const h8 xh = *reinterpret_cast<const h8*>(Ar + am_chunk(ar, c));
            const h8 xl = *reinterpret_cast<const h8*>(Ar + am_chunk(ar, 4 + c));
            const h8 yh = *reinterpret_cast<const h8*>(Br + am_chunk(brow, c));
            const h8 yl = *reinterpret_cast<const h8*>(Br + am_chunk(brow, 4 + c));
            acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, yh, acc, 0, 0, 0);
            acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, yh, acc2, 0, 0, 0);
            acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, yl, acc3, 0, 0, 0);
          }
        }
      }
      ALT_ST(5);  // MFMAs
      __syncthreads();  // every MFMA wave has read the band: its region takes S
      ALT_ST(6);
      if (g < 6) {
        // register r holds S[query 32mi + (r&3) + 8(r>>2) + 4h][band pixel 32ni + m]
#pragma unroll
        for (int r = 0; r < 16; ++r)
          S[(32 * mi + (r & 3) + 8 * (r >> 2) + 4 * h) * AM_SLD + 32 * ni + m] = acc[r] + acc2[r] + acc3[r];
      }
#endif
      ALT_ST(7);  // S stores
      __syncthreads();
      ALT_ST(8);
      // every lane (query) picks the taps of its window in box rows r0 .. r0 + br - 1
#pragma unroll
      for (int j = 0; j < TPT; ++j) {
        const int t = g + 8 * j;
        if (t < NT) {
          const int iy = t / WD, ix = t - (t / WD) * WD;
          const int rr = oy0 + iy - r0;
          if ((unsigned)rr < (unsigned)cur.br) tap[j] = S[lane * AM_SLD + rr * cur.bw + ox0 + ix];
        }
      }
      ALT_ST(9);  // tap picks
      __syncthreads();  // S read: the region takes the next band (or the tap sums)
      ALT_ST(10);
    }
    // ---- tap sums -> LDS ts[q][t] (over the band region), then the bilinear binning
    float* ts = reinterpret_cast<float*>(Bs);
    // (beside them: each query's bilinear fractions, pixel and validity for the binning below)
    f32x4* qtab = reinterpret_cast<f32x4*>(ts + AT * AT * (NT + 1));
#pragma unroll
    for (int j = 0; j < TPT; ++j) {
      const int t = g + 8 * j;
      if (t < NT) ts[lane * (NT + 1) + t] = tap[j];
    }
    if (g == 0)
      qtab[lane] = f32x4{cur.x - floorf(cur.x), cur.y - floorf(cur.y), __int_as_float(p), valid ? 1.f : 0.f};
    __syncthreads();
    ALT_ST(11);  // tap sums -> LDS + sync
    // bin (core/corr.py + correlation_kernel.cu:95-116: the bilinear weights of frac(coords) over
    // each bin's four integer taps, then / scale), the arithmetic of alt_bin_store
    const float sdiv = a0.scale_div;
    int big = 0;
    if (a0.out_layout == 1) {
      // thread t: outputs i = t + 512k of the tile's 64 x RD^2 (query i / RD^2, bin i % RD^2), all
      // independent (consecutive threads write consecutive bins of a query's row)
      constexpr int NO = AT * AT * RD * RD, KO = (NO + 511) / 512;
#pragma unroll 2
      for (int k = 0; k < KO; ++k) {
        const int i = tid + 512 * k;
        if (i < NO) {
          const int q = i / (RD * RD), o = i - q * (RD * RD);
          const f32x4 qi = qtab[q];
          if (qi[3] != 0.f) {
            const float dx = qi[0], dy = qi[1];
            const float* tq = ts + q * (NT + 1);
            const int ox = o / RD, oy = o - ox * RD;  // channel = oy + rd*ox
            float val = tq[oy * WD + ox] * ((1.f - dy) * (1.f - dx));
            val += tq[oy * WD + ox + 1] * ((1.f - dy) * dx);
            val += tq[(oy + 1) * WD + ox] * (dy * (1.f - dx));
            val += tq[(oy + 1) * WD + ox + 1] * (dy * dx);
            val = val / sdiv;
            big |= fabsf(val) > RAFT_RANGE_LIMIT;
            out[((long)b * P1 + __float_as_int(qi[2])) * a0.out_ld + o] = val;
          }
        }
      }
    } else if (valid) {
      // lanes = queries, wave g: bins o = g + 8i ([B][N][RD^2][H1][W1])
      const float dx = cur.x - floorf(cur.x), dy = cur.y - floorf(cur.y);
      const float* tq = ts + lane * (NT + 1);
      for (int o = g; o < RD * RD; o += 8) {
        const int ox = o / RD, oy = o - ox * RD;
        float val = tq[oy * WD + ox] * ((1.f - dy) * (1.f - dx));
        val += tq[oy * WD + ox + 1] * ((1.f - dy) * dx);
        val += tq[(oy + 1) * WD + ox] * (dy * (1.f - dx));
        val += tq[(oy + 1) * WD + ox + 1] * (dy * dx);
        val = val / sdiv;
        big |= fabsf(val) > RAFT_RANGE_LIMIT;
        out[(bn * (RD * RD) + o) * P1 + p] = val;
      }
    }
    ALT_ST(13);  // binning + output stores
    // the next level's box and first band go out behind this level's output stores (ahead of
    // them they held the stores back in the memory pipeline: 0.3-2 % slower, r04h_experiments)
    if (l + 1 < lvs.n) {
      setup(l + 1, nxt);
      if (nxt.fits) load_band(l + 1, nxt, 0);
    }
    ALT_ST(12);  // next level setup + first band issue
    if (a0.range_flag && big) *a0.range_flag = 1;
    if (valid && l == 0 && a0.flow && g == 0) {
      a0.flow[((long)b * P1 + p) * a0.flow_ld + 0] = cur.x * cdiv - (float)(p % a0.W1);
      a0.flow[((long)b * P1 + p) * a0.flow_ld + 1] = cur.y * cdiv - (float)(p / a0.W1);
    }
    __syncthreads();  // the tap sums are read: the band region takes the next level
    ALT_ST(14);  // flags, flow, final sync
    cur = nxt;
  }
#ifdef ALT_STAMPS
  if (lane == 0 && blockIdx.x < 4096) {
    unsigned long long* gs = g_altstamp + ((long)blockIdx.x * 8 + g) * 24;
    for (int k = 0; k < 16; ++k) gs[k] = alt_t[k];
    gs[16] = alt_clock() - alt_start;
    gs[17] = (unsigned long long)alt_bands;
  }
#endif
}


// Any radius (the reference's CorrBlock / AlternateCorrBlock take any r; RAFT uses 3 and 4,
// which the kernels above serve): one wave per query, the (2r+2)^2 tap sums in dynamic LDS
// (one row of ALT_GEN_ROW floats per wave), then the bilinear binning.
__global__ __launch_bounds__(256) void alt_corr_generic_kernel(AltArgs a, int row) {
  extern __shared__ float gts[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const int P1 = a.H1 * a.W1;
  const long gid = (long)blockIdx.x * 4 + wv;
  if (gid >= (long)a.B * a.N * P1) return;
  const long bn = gid / P1;
  const int p = (int)(gid - bn * P1);
  const int b = (int)(bn / a.N);
  const int rd = 2 * a.r + 1, wd = 2 * a.r + 2;
  float* ts = gts + wv * row;
  float x, y;
  if (a.coords_layout == 0) {
    x = a.coords[2 * gid];
    y = a.coords[2 * gid + 1];
  } else {
    x = a.coords[((long)b * 2) * P1 + p];
    y = a.coords[((long)b * 2 + 1) * P1 + p];
  }
  x = x / a.coord_div;
  y = y / a.coord_div;
  const bool fin = isfinite(x) && isfinite(y) && fabsf(x) < 1e8f && fabsf(y) < 1e8f;
  const int x0 = fin ? (int)floorf(x) - a.r : 0, y0 = fin ? (int)floorf(y) - a.r : 0;
  const float* f1row = a.f1 + ((long)b * P1 + p) * a.C;
  const float* f2b = a.f2 + (long)b * a.H2 * a.W2 * a.C;
  for (int t = 0; t < wd * wd; ++t) {
    const int h2 = y0 + t / wd, w2 = x0 + t % wd;
    float v = 0.f;
    if ((unsigned)h2 < (unsigned)a.H2 && (unsigned)w2 < (unsigned)a.W2) {
      const float* r2 = f2b + ((long)h2 * a.W2 + w2) * a.C;
      for (int c = 4 * lane; c < a.C; c += 256) {
        const f32x4 u = *reinterpret_cast<const f32x4*>(r2 + c);
        const f32x4 f = *reinterpret_cast<const f32x4*>(f1row + c);
        v += f[0] * u[0] + f[1] * u[1] + f[2] * u[2] + f[3] * u[3];
      }
    }
#pragma unroll
    for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
    if (lane == 0) ts[t] = v;
  }
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  const float dx = x - floorf(x), dy = y - floorf(y);
  for (int o = lane; o < rd * rd; o += 64) {
    const int ox = o / rd, oy = o - ox * rd;  // channel = oy + rd*ox
    float val = ts[oy * wd + ox] * ((1.f - dy) * (1.f - dx));
    val += ts[oy * wd + ox + 1] * ((1.f - dy) * dx);
    val += ts[(oy + 1) * wd + ox] * (dy * (1.f - dx));
    val += ts[(oy + 1) * wd + ox + 1] * (dy * dx);
    val = val / a.scale_div;
    if (a.range_flag && fabsf(val) > RAFT_RANGE_LIMIT) *a.range_flag = 1;
    if (a.out_layout == 0)
      a.out[(bn * (rd * rd) + o) * P1 + p] = val;
    else
      a.out[((long)b * P1 + p) * a.out_ld + o] = val;
  }
  if (a.flow && lane < 2) {
    const float gx = lane == 0 ? (float)(p % a.W1) : (float)(p / a.W1);
    a.flow[((long)b * P1 + p) * a.flow_ld + lane] = (lane == 0 ? x : y) * a.coord_div - gx;
  }
}

int launch_alt(const AltArgs& a, raft_stream_t stream) {
  hipStream_t s = as_stream(stream);
  if (a.r > 4) {  // any radius: the generic kernel
    const int wd = 2 * a.r + 2, row = wd * wd;
    const long waves = (long)a.B * a.N * a.H1 * a.W1;
    hipLaunchKernelGGL(alt_corr_generic_kernel, dim3((unsigned)cdiv_l(waves, 4)), dim3(256),
                       (size_t)(4 * row * sizeof(float)), s, a, row);
    return check_launch("raft_alt_corr(generic radius)");
  }
#ifndef ALT_NO_TILE  // dev builds: the per-pixel kernel at every size
  static const bool mfma = [] {
    const char* e = getenv("RAFT_ALT_MFMA");
    return !(e && e[0] == '0');
  }();
  if (mfma && a.prec != RAFT_PREC_FP32 && a.r == 4 && a.C % 32 == 0 && a.C <= 256) {
    const long tiles = (long)a.B * a.N * cdiv_l(a.H1, AT) * cdiv_l(a.W1, AT);
    AltLevels lv{};
    lv.f2[0] = a.f2;
    lv.out[0] = a.out;
    lv.H2[0] = a.H2;
    lv.W2[0] = a.W2;
    lv.div[0] = a.coord_div;
    lv.n = 1;
    hipLaunchKernelGGL(alt_corr_mfma_kernel<4>, dim3((unsigned)tiles), dim3(512), 0, s, a, lv);
    return check_launch("raft_alt_corr(mfma)");
  }
  if (a.r == 4 && a.C % ACC == 0 && a.C <= 256) {
    const long tiles = (long)a.B * a.N * cdiv_l(a.H1, AT) * cdiv_l(a.W1, AT);
    hipLaunchKernelGGL(alt_corr_tile_kernel<4>, dim3((unsigned)tiles), dim3(256), 0, s, a);
    return check_launch("raft_alt_corr");
  }
#endif
  const long waves = (long)a.B * a.N * a.H1 * a.W1;
  dim3 grid((unsigned)cdiv_l(waves, 4));
  if (a.C <= 256)
    hipLaunchKernelGGL(alt_corr_kernel<1>, grid, dim3(256), 0, s, a);
  else if (a.C <= 512)
    hipLaunchKernelGGL(alt_corr_kernel<2>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(alt_corr_kernel<4>, grid, dim3(256), 0, s, a);
  return check_launch("raft_alt_corr");
}

__global__ void avgpool2_nhwc_kernel(const float* in, float* out, int B, int H, int W, int C, int Ho, int Wo) {
  const long total = (long)B * Ho * Wo * C;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int c = i % C;
    long t = i / C;
    const int x = t % Wo;
    t /= Wo;
    const int y = t % Ho;
    const int b = t / Ho;
    const float* p = in + (((long)b * H + 2 * y) * W + 2 * x) * C + c;
    out[i] = (((p[0] + p[C]) + p[(long)W * C]) + p[(long)W * C + C]) / 4.0f;
  }
}

}  // namespace

#ifdef ALT_STAMPS
extern "C" int raft_debug_altstamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_altstamp), sizeof(unsigned long long) * (size_t)n);
}
#endif
}  // namespace raft

using namespace raft;

static int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

static int alt_checks(const float* f1, const float* f2, const float* coords, const float* out, int B, int H1, int W1,
                      int H2, int W2, int C, int N, int r) {
  RAFT_REQUIRE(f1 && f2 && coords && out, "raft_alt_corr: null pointer");
  RAFT_REQUIRE(B > 0 && H1 > 0 && W1 > 0 && H2 > 0 && W2 > 0 && C > 0 && N > 0, "raft_alt_corr: bad sizes");
  RAFT_REQUIRE(C % 4 == 0 && C <= 1024, "raft_alt_corr: C must be a multiple of 4 and <= 1024 (got %d)", C);
  RAFT_REQUIRE(r >= 0 && r <= 32, "raft_alt_corr: radius must be 0..32 (got %d)", r);
  RAFT_REQUIRE((((uintptr_t)f1 | (uintptr_t)f2) & 15) == 0, "raft_alt_corr: fmaps must be 16-byte aligned");
  RAFT_REQUIRE((long)H2 * W2 * C * 4 < (1L << 31), "raft_alt_corr: one fmap2 exceeds 2 GiB");
  return 0;
}

extern "C" int raft_alt_corr_forward(const float* fmap1, const float* fmap2, const float* coords, float* corr, int B,
                                     int H1, int W1, int H2, int W2, int C, int N, int radius, float scale_div,
                                     raft_stream_t stream) {
  // the plugin's contract is the reference kernel's exact fp32 arithmetic
  return raft_alt_corr_forward_prec(fmap1, fmap2, coords, corr, B, H1, W1, H2, W2, C, N, radius, scale_div,
                                    RAFT_PREC_FP32, stream);
}

extern "C" int raft_alt_corr_forward_prec(const float* fmap1, const float* fmap2, const float* coords, float* corr,
                                          int B, int H1, int W1, int H2, int W2, int C, int N, int radius,
                                          float scale_div, int precision, raft_stream_t stream) {
  int rc = alt_checks(fmap1, fmap2, coords, corr, B, H1, W1, H2, W2, C, N, radius);
  if (rc) return rc;
  AltArgs a;
  a.f1 = fmap1;
  a.f2 = fmap2;
  a.coords = coords;
  a.coords_layout = 0;
  a.coord_div = 1.0f;
  a.out = corr;
  a.out_layout = 0;
  a.out_ld = 0;
  a.B = B;
  a.H1 = H1;
  a.W1 = W1;
  a.H2 = H2;
  a.W2 = W2;
  a.C = C;
  a.N = N;
  a.r = radius;
  a.scale_div = scale_div;
  a.flow = nullptr;
  a.flow_ld = 0;
  a.range_flag = nullptr;
  a.prec = precision;
  return launch_alt(a, stream);
}

extern "C" int raft_alt_corr_lookup_nhwc(const float* fmap1, const float* fmap2, const float* coords,
                                         int coords_layout, float coord_div, float* out, int out_ld, int B, int H1,
                                         int W1, int H2, int W2, int C, int radius, float scale_div, float* flow_out,
                                         int flow_ld, int* range_flag, raft_stream_t stream) {
  return raft_alt_corr_lookup_nhwc_prec(fmap1, fmap2, coords, coords_layout, coord_div, out, out_ld, B, H1, W1, H2, W2,
                                        C, radius, scale_div, flow_out, flow_ld, range_flag, RAFT_PREC_F16X3, stream);
}

extern "C" int raft_alt_corr_lookup_nhwc_prec(const float* fmap1, const float* fmap2, const float* coords,
                                              int coords_layout, float coord_div, float* out, int out_ld, int B,
                                              int H1, int W1, int H2, int W2, int C, int radius, float scale_div,
                                              float* flow_out, int flow_ld, int* range_flag, int precision,
                                              raft_stream_t stream) {
  int rc = alt_checks(fmap1, fmap2, coords, out, B, H1, W1, H2, W2, C, 1, radius);
  if (rc) return rc;
  RAFT_REQUIRE(coords_layout == 0 || coords_layout == 1, "raft_alt_corr_lookup_nhwc: bad coords_layout");
  RAFT_REQUIRE(coord_div > 0.f, "raft_alt_corr_lookup_nhwc: coord_div must be > 0");
  RAFT_REQUIRE(out_ld >= (2 * radius + 1) * (2 * radius + 1), "raft_alt_corr_lookup_nhwc: out_ld too small");
  AltArgs a;
  a.f1 = fmap1;
  a.f2 = fmap2;
  a.coords = coords;
  a.coords_layout = coords_layout;
  a.coord_div = coord_div;
  a.out = out;
  a.out_layout = 1;
  a.out_ld = out_ld;
  a.B = B;
  a.H1 = H1;
  a.W1 = W1;
  a.H2 = H2;
  a.W2 = W2;
  a.C = C;
  a.N = 1;
  a.r = radius;
  a.scale_div = scale_div;
  a.flow = flow_out;
  a.flow_ld = flow_ld;
  a.range_flag = range_flag;
  a.prec = precision;
  return launch_alt(a, stream);
}

extern "C" int raft_alt_corr_lookup_levels(const float* fmap1, const float* const* fmap2_levels, const int* h2s,
                                           const int* w2s, int L, const float* coords, int coords_layout, float* out,
                                           int out_ld, int B, int H1, int W1, int C, int radius, float scale_div,
                                           float* flow_out, int flow_ld, int* range_flag, raft_stream_t stream) {
  return raft_alt_corr_lookup_levels_prec(fmap1, fmap2_levels, h2s, w2s, L, coords, coords_layout, out, out_ld, B, H1,
                                          W1, C, radius, scale_div, flow_out, flow_ld, range_flag, RAFT_PREC_F16X3,
                                          stream);
}

extern "C" int raft_alt_corr_lookup_levels_prec(const float* fmap1, const float* const* fmap2_levels, const int* h2s,
                                                const int* w2s, int L, const float* coords, int coords_layout,
                                                float* out, int out_ld, int B, int H1, int W1, int C, int radius,
                                                float scale_div, float* flow_out, int flow_ld, int* range_flag,
                                                int precision, raft_stream_t stream) {
  RAFT_REQUIRE(fmap2_levels && h2s && w2s && L >= 1 && L <= AM_MAXL,
               "raft_alt_corr_lookup_levels: need 1..%d levels", AM_MAXL);
  const int rd2 = (2 * radius + 1) * (2 * radius + 1);
  RAFT_REQUIRE(out_ld >= L * rd2, "raft_alt_corr_lookup_levels: out_ld too small for %d levels", L);
  for (int l = 0; l < L; ++l) {
    int rc = alt_checks(fmap1, fmap2_levels[l], coords, out, B, H1, W1, h2s[l], w2s[l], C, 1, radius);
    if (rc) return rc;
  }
  RAFT_REQUIRE(coords_layout == 0 || coords_layout == 1, "raft_alt_corr_lookup_levels: bad coords_layout");
  static const bool mfma = [] {
    const char* e = getenv("RAFT_ALT_MFMA");
    return !(e && e[0] == '0');
  }();
  if (!(mfma && precision != RAFT_PREC_FP32 && radius == 4 && C % 32 == 0 && C <= 256)) {
    // one launch per level (raft_alt_corr_lookup_nhwc_prec; the flow is written with level 0)
    for (int l = 0; l < L; ++l) {
      int rc = raft_alt_corr_lookup_nhwc_prec(fmap1, fmap2_levels[l], coords, coords_layout, (float)(1 << l),
                                              out + (long)l * rd2, out_ld, B, H1, W1, h2s[l], w2s[l], C, radius,
                                              scale_div, l == 0 ? flow_out : nullptr, flow_ld, range_flag, precision,
                                              stream);
      if (rc) return rc;
    }
    return 0;
  }
  AltArgs a;
  a.f1 = fmap1;
  a.f2 = fmap2_levels[0];
  a.coords = coords;
  a.coords_layout = coords_layout;
  a.coord_div = 1.f;
  a.out = out;
  a.out_layout = 1;
  a.out_ld = out_ld;
  a.B = B;
  a.H1 = H1;
  a.W1 = W1;
  a.H2 = h2s[0];
  a.W2 = w2s[0];
  a.C = C;
  a.N = 1;
  a.r = radius;
  a.scale_div = scale_div;
  a.flow = flow_out;
  a.flow_ld = flow_ld;
  a.range_flag = range_flag;
  a.prec = precision;
  AltLevels lv{};
  for (int l = 0; l < L; ++l) {
    lv.f2[l] = fmap2_levels[l];
    lv.out[l] = out + (long)l * rd2;
    lv.H2[l] = h2s[l];
    lv.W2[l] = w2s[l];
    lv.div[l] = (float)(1 << l);
  }
  lv.n = L;
  const long tiles = (long)B * cdiv_l(H1, AT) * cdiv_l(W1, AT);
  hipLaunchKernelGGL(alt_corr_mfma_kernel<4>, dim3((unsigned)tiles), dim3(512), 0, as_stream(stream), a, lv);
  return check_launch("raft_alt_corr_lookup_levels");
}

extern "C" int raft_avgpool2_nhwc(const float* in, float* out, int B, int H, int W, int C, raft_stream_t stream) {
  RAFT_REQUIRE(in && out && B > 0 && H >= 2 && W >= 2 && C > 0, "raft_avgpool2_nhwc: bad arguments");
  const int Ho = H / 2, Wo = W / 2;
  const long n = (long)B * Ho * Wo * C;
  hipLaunchKernelGGL(avgpool2_nhwc_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), in, out, B, H, W, C,
                     Ho, Wo);
  return check_launch("raft_avgpool2_nhwc");
}
