// Correlation kernels for gfx950: all-pairs volume + pyramid, radius-r window
// lookup, and the on-the-fly ("alternate") correlation of alt_cuda_corr.
#include "common.hpp"

namespace raft {
namespace {

// ============================================================================
// K2: all-pairs correlation volume + pyramid levels 0 and 1
//     (CorrBlock.corr core/corr.py:96-127 and CorrBlock.__init__ :25-54)
//
// GEMM per batch b: C[p1, p2] = <fmap1[p1], fmap2[p2]> / sqrt_c, M = N = H*W,
// K = C.  The N tile is a 2-row x 32-column patch of the (h2, w2) grid, so
// one tile holds whole 2x2 pooling windows (level 1 comes out of the same
// epilogue) and its level-0 rows are 128-B contiguous runs of the
// [p1][H][W] map.  Levels >= 2 are pooled from level 1 by pool2_kernel.
// ============================================================================
constexpr int CB_BM = 64, CB_BN = 64, CB_BK = 32, CB_LDSK = CB_BK + 4;
constexpr int CB_TW = 32;  // tile width in w2 (2 rows of 32)

struct CorrBuildArgs {
  const float* f1;
  const float* f2;
  int ld, H, W, C, P;
  float sqrt_c;
  float* lvl0;  // [B][P][H][W]
  float* lvl1;  // [B][P][H/2][W/2] or null
  int H1, W1;
  int ntw;      // tiles along w2
};

__global__ __launch_bounds__(256) void corr_build_kernel(CorrBuildArgs a) {
  constexpr int STAGE = (CB_BM + CB_BN) * CB_LDSK;
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int b = blockIdx.z;
  const int m0 = blockIdx.x * CB_BM;
  const int th = blockIdx.y / a.ntw;   // row pair index
  const int tw = blockIdx.y - th * a.ntw;
  const int h2base = 2 * th, w2base = tw * CB_TW;

  const int lr = tid >> 3, lq = tid & 7;
  const float* arow[2];
  const float* brow[2];
  bool av_[2], bv_[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = lr + 32 * i;
    const int p1 = m0 + r;
    av_[i] = p1 < a.P;
    arow[i] = a.f1 + ((long)b * a.P + (av_[i] ? p1 : 0)) * a.ld + lq * 4;
    const int h2 = h2base + (r >> 5), w2 = w2base + (r & 31);
    bv_[i] = h2 < a.H && w2 < a.W;
    brow[i] = a.f2 + ((long)b * a.P + (bv_[i] ? h2 * a.W + w2 : 0)) * a.ld + lq * 4;
  }
  f32x4 ra[2], rb[2];
  auto gload = [&](int kc) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const f32x4 z = {0.f, 0.f, 0.f, 0.f};
      const bool cin = kc * CB_BK + lq * 4 < a.C;  // C % 4 == 0; zero-fill the K tail
      ra[i] = (av_[i] && cin) ? *reinterpret_cast<const f32x4*>(arow[i] + kc * CB_BK) : z;
      rb[i] = (bv_[i] && cin) ? *reinterpret_cast<const f32x4*>(brow[i] + kc * CB_BK) : z;
    }
  };
  auto sstore = [&](int buf) {
    float* A = smem + buf * STAGE;
    float* Bt = A + CB_BM * CB_LDSK;
    *reinterpret_cast<f32x4*>(A + lr * CB_LDSK + lq * 4) = ra[0];
    *reinterpret_cast<f32x4*>(A + (lr + 32) * CB_LDSK + lq * 4) = ra[1];
    *reinterpret_cast<f32x4*>(Bt + lr * CB_LDSK + lq * 4) = rb[0];
    *reinterpret_cast<f32x4*>(Bt + (lr + 32) * CB_LDSK + lq * 4) = rb[1];
  };
  const int nk = cdiv(a.C, CB_BK);
  gload(0);
  sstore(0);
  __syncthreads();
  f32x16 acc = {};
  const int ao = (wm * 32 + (lane & 31)) * CB_LDSK + (lane >> 5) * 16;
  const int bo = (wn * 32 + (lane & 31)) * CB_LDSK + (lane >> 5) * 16;
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    const bool more = kc + 1 < nk;
    if (more) gload(kc + 1);
    const float* A = smem + cur * STAGE;
    const float* Bt = A + CB_BM * CB_LDSK;
    f32x4 x[4], y[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      x[j] = *reinterpret_cast<const f32x4*>(A + ao + 4 * j);
      y[j] = *reinterpret_cast<const f32x4*>(Bt + bo + 4 * j);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s)
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s >> 2][s & 3], y[s >> 2][s & 3], acc, 0, 0, 0);
    if (more) sstore(cur ^ 1);
    __syncthreads();
  }

  // epilogue: scaled tile -> LDS T[64 p1][64 (h2 row 0: 0..31 | row 1: 32..63)]
  constexpr int TLD = CB_BN + 1;
  float* T = smem;
  {
    const int n = wn * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      T[row * TLD + n] = acc[r] / a.sqrt_c;
    }
  }
  __syncthreads();
  const long HW = (long)a.H * a.W;
  for (int idx = tid; idx < CB_BM * CB_BN; idx += 256) {
    const int row = idx >> 6, n = idx & 63;
    const int p1 = m0 + row;
    const int h2 = h2base + (n >> 5), w2 = w2base + (n & 31);
    if (p1 < a.P && h2 < a.H && w2 < a.W)
      a.lvl0[((long)b * a.P + p1) * HW + (long)h2 * a.W + w2] = T[row * TLD + n];
  }
  if (a.lvl1) {
    const long HW1 = (long)a.H1 * a.W1;
    const int y1 = th;
    for (int idx = tid; idx < CB_BM * (CB_TW / 2); idx += 256) {
      const int row = idx >> 4, j = idx & 15;
      const int p1 = m0 + row;
      const int x1 = (w2base >> 1) + j;
      if (p1 < a.P && y1 < a.H1 && x1 < a.W1) {
        const float* t = T + row * TLD;
        const float s = ((t[2 * j] + t[2 * j + 1]) + t[32 + 2 * j]) + t[32 + 2 * j + 1];
        a.lvl1[((long)b * a.P + p1) * HW1 + (long)y1 * a.W1 + x1] = s / 4.0f;
      }
    }
  }
}

// 2x2 / stride-2 average pool over the last two dims of [N][H][W] (floor),
// summation order of the reference's CPU avg_pool2d (row-major window).
__global__ void pool2_kernel(const float* __restrict__ in, float* __restrict__ out, long n_maps, int H, int W,
                             int Ho, int Wo) {
  const long total = n_maps * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = i % Wo;
    const long t = i / Wo;
    const int y = t % Ho;
    const long n = t / Ho;
    const float* p = in + (n * H + 2 * y) * W + 2 * x;
    out[i] = (((p[0] + p[1]) + p[W]) + p[W + 1]) / 4.0f;
  }
}

// ============================================================================
// K1: radius-r lookup of every pyramid level (CorrBlock.__call__ core/corr.py:56-94)
//
// One wave per query pixel.  Phase 1: the wave stages the (2r+2)^2 integer
// window around floor(coords/2^l) - r of every level into LDS (zero outside
// the map).  Phase 2: each lane evaluates taps of the (2r+1)^2 x L output
// with the reference's arithmetic (offset added to the centroid, then
// bilinear_sampler's normalise 2x/(W-1)-1 and grid_sample's unnormalise
// (x+1)*((W-1)/2)), so every tap's corner indices and weights are the ones
// the reference computes; corners come from the LDS window (or, when the
// float round trip moved a tap's floor off the window, from global memory).
// Output channel = lvl*(2r+1)^2 + ix*(2r+1) + iy (x-major), contiguous per pixel.
// ============================================================================
constexpr int LK_MAXL = 6;

struct LookupArgs {
  const float* pyr;
  long lvl_off[LK_MAXL];
  int lh[LK_MAXL], lw[LK_MAXL];
  int B, H, W, L, r;
  const float* coords;
  int coords_layout;
  float* out;
  int out_ld, out_layout;
  float* flow;
  int flow_ld;
};

__device__ __forceinline__ void load_coords(const float* c, int layout, int b, int p, int P, float& x, float& y) {
  if (layout == 0) {
    x = c[2L * ((long)b * P + p)];
    y = c[2L * ((long)b * P + p) + 1];
  } else {
    x = c[((long)b * 2) * P + p];
    y = c[((long)b * 2 + 1) * P + p];
  }
}

template <int R>
__global__ __launch_bounds__(256) void corr_lookup_kernel(LookupArgs a) {
  constexpr int RD = 2 * R + 1;
  constexpr int WD = 2 * R + 2;
  constexpr int WIN = WD * WD;
  __shared__ float win[4][LK_MAXL][WIN];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int P = a.H * a.W;
  const long gp = (long)blockIdx.x * 4 + wv;  // global pixel index b*P + p
  const bool valid = gp < (long)a.B * P;
  const int b = valid ? (int)(gp / P) : 0;
  const int p = valid ? (int)(gp - (long)b * P) : 0;
  float x = 0.f, y = 0.f;
  if (valid) load_coords(a.coords, a.coords_layout, b, p, P, x, y);

  // phase 1: stage windows
  for (int l = 0; l < a.L; ++l) {
    const float s = 1.0f / (float)(1 << l);   // coords / 2**l (exact power-of-two scaling)
    const int x0 = (int)floorf(x * s) - R, y0 = (int)floorf(y * s) - R;
    const int Hl = a.lh[l], Wl = a.lw[l];
    const float* map = a.pyr + a.lvl_off[l] + gp * (long)Hl * Wl;
    for (int e = lane; e < WIN; e += 64) {
      const int wy = e / WD, wx = e - wy * WD;
      const int yy = y0 + wy, xx = x0 + wx;
      float v = 0.f;
      if (valid && yy >= 0 && yy < Hl && xx >= 0 && xx < Wl) v = map[(long)yy * Wl + xx];
      win[wv][l][e] = v;
    }
  }
  __syncthreads();
  if (!valid) return;

  // phase 2: taps
  const int ntap = a.L * RD * RD;
  for (int t = lane; t < ntap; t += 64) {
    const int l = t / (RD * RD);
    const int tt = t - l * RD * RD;
    const int ix = tt / RD, iy = tt - ix * RD;
    const float s = 1.0f / (float)(1 << l);
    const float cx = x * s, cy = y * s;
    const int Hl = a.lh[l], Wl = a.lw[l];
    const int x0w = (int)floorf(cx) - R, y0w = (int)floorf(cy) - R;
    // reference arithmetic: centroid + delta, normalise, unnormalise
    const float X = cx + (float)(ix - R);
    const float Y = cy + (float)(iy - R);
    const float wm1 = (float)(Wl - 1), hm1 = (float)(Hl - 1);
    const float gx = 2.0f * X / wm1 - 1.0f;
    const float gy = 2.0f * Y / hm1 - 1.0f;
    const float ux = (gx + 1.0f) * (wm1 / 2.0f);
    const float uy = (gy + 1.0f) * (hm1 / 2.0f);
    float v;
    if (!(isfinite(ux) && isfinite(uy))) {
      v = __builtin_nanf("");
    } else {
      const float fx0 = floorf(ux), fy0 = floorf(uy);
      const float tx = ux - fx0, ty = uy - fy0;
      const int xi = (int)fx0, yi = (int)fy0;
      const int wx = xi - x0w, wy = yi - y0w;
      float vnw, vne, vsw, vse;
      if (wx >= 0 && wx + 1 < WD && wy >= 0 && wy + 1 < WD) {
        const float* w = win[wv][l] + wy * WD + wx;
        vnw = w[0];
        vne = w[1];
        vsw = w[WD];
        vse = w[WD + 1];
      } else {
        const float* map = a.pyr + a.lvl_off[l] + gp * (long)Hl * Wl;
        auto at = [&](int yy, int xx) {
          return (yy >= 0 && yy < Hl && xx >= 0 && xx < Wl) ? map[(long)yy * Wl + xx] : 0.f;
        };
        vnw = at(yi, xi);
        vne = at(yi, xi + 1);
        vsw = at(yi + 1, xi);
        vse = at(yi + 1, xi + 1);
      }
      const float e = 1.0f - tx, sS = 1.0f - ty;
      v = vnw * (sS * e) + vne * (sS * tx) + vsw * (ty * e) + vse * (ty * tx);
    }
    if (a.out_layout == 0)
      a.out[gp * a.out_ld + t] = v;
    else
      a.out[((long)b * ntap + t) * P + p] = v;
  }
  if (a.flow && lane < 2) {
    const float g = lane == 0 ? (float)(p % a.W) : (float)(p / a.W);
    a.flow[gp * a.flow_ld + lane] = (lane == 0 ? x : y) - g;
  }
}

// ============================================================================
// K3: on-the-fly correlation (alt_cuda_corr forward, correlation_kernel.cu:18-119)
//
// One wave per (query pixel, coordinate set).  fmap1[p] is held in registers,
// 4 channels per lane per 256-channel slab.  The (2r+2)^2 integer taps
// around floor(coords) - r are visited 64 at a time: every lane reads the
// tap's fmap2 row slice (one coalesced 1 KiB read per tap per slab) and keeps
// a private partial dot product per tap; a transposing butterfly (halving
// exchange, 63 shuffles per 64 taps) leaves lane j holding tap j's full sum.
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
};

template <int NV>
__device__ __forceinline__ float tap_partial(const f32x4 (&f1)[NV], const float* row, int lane, int C) {
  float s = 0.f;
#pragma unroll
  for (int k = 0; k < NV; ++k) {
    const int c = k * 256 + lane * 4;
    if (c < C) {
      const f32x4 v = *reinterpret_cast<const f32x4*>(row + c);
      s += f1[k][0] * v[0] + f1[k][1] * v[1] + f1[k][2] * v[2] + f1[k][3] * v[3];
    }
  }
  return s;
}

// Reduce v[0..63] (one partial per tap, per lane) so that lane j ends with sum over lanes of v[j].
__device__ __forceinline__ float transpose_reduce64(float (&v)[64], int lane) {
#pragma unroll
  for (int half = 32; half >= 1; half >>= 1) {
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

template <int NV>
__global__ __launch_bounds__(256) void alt_corr_kernel(AltArgs a) {
  __shared__ float tapsum[4][128];
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int P1 = a.H1 * a.W1;
  const long gid = (long)blockIdx.x * 4 + wv;  // ((b*N + n)*P1 + p)
  const bool valid = gid < (long)a.B * a.N * P1;
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
  for (int g = 0; g < ntaps; g += 64) {
    float v[64];
#pragma unroll
    for (int j = 0; j < 64; ++j) {
      const int t = g + j;
      const int iy = t / wd, ix = t - iy * wd;
      const int h2 = y0 + iy, w2 = x0 + ix;
      float s = 0.f;
      if (valid && t < ntaps && h2 >= 0 && h2 < a.H2 && w2 >= 0 && w2 < a.W2)
        s = tap_partial<NV>(f1, f2b + ((long)h2 * a.W2 + w2) * a.C, lane, a.C);
      v[j] = s;
    }
    const float tot = transpose_reduce64(v, lane);
    if (g + lane < ntaps) tapsum[wv][g + lane] = tot;
  }
  __syncthreads();
  if (!valid) return;
  for (int o = lane; o < rd * rd; o += 64) {
    const int ox = o / rd, oy = o - ox * rd;  // channel = oy + rd*ox
    const float* ts = tapsum[wv];
    const float s00 = ts[oy * wd + ox], s01 = ts[oy * wd + ox + 1];
    const float s10 = ts[(oy + 1) * wd + ox], s11 = ts[(oy + 1) * wd + ox + 1];
    float val = s00 * ((1.f - dy) * (1.f - dx));
    val += s01 * ((1.f - dy) * dx);
    val += s10 * (dy * (1.f - dx));
    val += s11 * (dy * dx);
    val = val / a.scale_div;
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
  const long waves = (long)a.B * a.N * a.H1 * a.W1;
  dim3 grid((unsigned)cdiv_l(waves, 4));
  hipStream_t s = as_stream(stream);
  if (a.C <= 256)
    hipLaunchKernelGGL(alt_corr_kernel<1>, grid, dim3(256), 0, s, a);
  else if (a.C <= 512)
    hipLaunchKernelGGL(alt_corr_kernel<2>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(alt_corr_kernel<4>, grid, dim3(256), 0, s, a);
  return check_launch("raft_alt_corr");
}

// ---------------------------------------------------------------------------
// alt backward (training path, correlation_kernel.cu:122-256):
// g(tap) = sum of the corr_grad bins the tap fed, weighted as in forward;
// fmap1_grad[p] = sum_tap g * fmap2[tap] (gather, deterministic);
// fmap2_grad[q] += g * fmap1[p] (float atomics, as the reference).
// ---------------------------------------------------------------------------
__global__ __launch_bounds__(256) void alt_corr_bwd_kernel(const float* f1, const float* f2, const float* coords,
                                                         const float* cg, float* f1g, float* f2g, int B, int H1,
                                                         int W1, int H2, int W2, int C, int N, int r) {
  const int lane = threadIdx.x & 63;
  const int wv = threadIdx.x >> 6;
  const int P1 = H1 * W1;
  const long gid = (long)blockIdx.x * 4 + wv;  // b*P1 + p
  if (gid >= (long)B * P1) return;
  const int b = (int)(gid / P1);
  const int p = (int)(gid - (long)b * P1);
  const int rd = 2 * r + 1, wd = 2 * r + 2;
  for (int c0 = lane * 4; c0 < C; c0 += 256) {
    f32x4 acc1 = {0.f, 0.f, 0.f, 0.f};
    const f32x4 a1 = *reinterpret_cast<const f32x4*>(f1 + gid * C + c0);
    for (int n = 0; n < N; ++n) {
      const long bn = (long)b * N + n;
      const float x = coords[2 * (bn * P1 + p)], y = coords[2 * (bn * P1 + p) + 1];
      const float fx = floorf(x), fy = floorf(y);
      const float dx = x - fx, dy = y - fy;
      const int x0 = (int)fx - r, y0 = (int)fy - r;
      const float* g = cg + bn * rd * rd * P1 + p;
      for (int iy = 0; iy < wd; ++iy) {
        for (int ix = 0; ix < wd; ++ix) {
          const int h2 = y0 + iy, w2 = x0 + ix;
          if (h2 < 0 || h2 >= H2 || w2 < 0 || w2 >= W2) continue;
          float gt = 0.f;
          if (iy > 0 && ix > 0) gt += g[(long)((iy - 1) + rd * (ix - 1)) * P1] * dy * dx;
          if (iy > 0 && ix < rd) gt += g[(long)((iy - 1) + rd * ix) * P1] * dy * (1.f - dx);
          if (iy < rd && ix > 0) gt += g[(long)(iy + rd * (ix - 1)) * P1] * (1.f - dy) * dx;
          if (iy < rd && ix < rd) gt += g[(long)(iy + rd * ix) * P1] * (1.f - dy) * (1.f - dx);
          float* q2 = f2g + (((long)b * H2 + h2) * W2 + w2) * C + c0;
          const f32x4 b2 = *reinterpret_cast<const f32x4*>(f2 + (((long)b * H2 + h2) * W2 + w2) * C + c0);
          acc1 += gt * b2;
#pragma unroll
          for (int j = 0; j < 4; ++j) atomicAdd(q2 + j, gt * a1[j]);
        }
      }
    }
    *reinterpret_cast<f32x4*>(f1g + gid * C + c0) = acc1;
  }
}

__global__ void zero_kernel(float* p, long n) {
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n; i += (long)gridDim.x * blockDim.x) p[i] = 0.f;
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
}  // namespace raft

using namespace raft;

static void pyramid_dims(int H, int W, int L, int* hs, int* ws) {
  hs[0] = H;
  ws[0] = W;
  for (int l = 1; l < L; ++l) {
    hs[l] = hs[l - 1] / 2;
    ws[l] = ws[l - 1] / 2;
  }
}

extern "C" size_t raft_corr_pyramid_floats(int B, int H, int W, int L) {
  if (B <= 0 || H <= 0 || W <= 0 || L <= 0 || L > LK_MAXL) return 0;
  int hs[LK_MAXL], ws[LK_MAXL];
  pyramid_dims(H, W, L, hs, ws);
  size_t tot = 0;
  for (int l = 0; l < L; ++l) tot += (size_t)hs[l] * ws[l];
  return tot * (size_t)B * H * W;
}

static int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

extern "C" int raft_corr_build(const float* fmap1, const float* fmap2, int ld, int B, int H, int W, int C, int L,
                               float sqrt_c, float* pyramid, raft_stream_t stream) {
  RAFT_REQUIRE(fmap1 && fmap2 && pyramid, "raft_corr_build: null pointer");
  RAFT_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && L >= 1 && L <= LK_MAXL, "raft_corr_build: bad sizes");
  RAFT_REQUIRE(C % 4 == 0, "raft_corr_build: C must be a multiple of 4 (got %d)", C);
  RAFT_REQUIRE(ld % 4 == 0 && ld >= C, "raft_corr_build: ld must be >= C and a multiple of 4");
  RAFT_REQUIRE((((uintptr_t)fmap1 | (uintptr_t)fmap2) & 15) == 0, "raft_corr_build: fmaps must be 16-byte aligned");
  int hs[LK_MAXL], ws[LK_MAXL];
  pyramid_dims(H, W, L, hs, ws);
  for (int l = 1; l < L; ++l)
    RAFT_REQUIRE(hs[l] >= 1 && ws[l] >= 1, "raft_corr_build: level %d is empty (%dx%d input)", l, H, W);
  const long P = (long)H * W;
  CorrBuildArgs a;
  a.f1 = fmap1;
  a.f2 = fmap2;
  a.ld = ld;
  a.H = H;
  a.W = W;
  a.C = C;
  a.P = (int)P;
  a.sqrt_c = sqrt_c;
  a.lvl0 = pyramid;
  a.H1 = hs[L > 1 ? 1 : 0];
  a.W1 = ws[L > 1 ? 1 : 0];
  a.lvl1 = L > 1 ? pyramid + (size_t)B * P * P : nullptr;
  a.ntw = cdiv(W, CB_TW);
  hipStream_t s = as_stream(stream);
  dim3 grid(cdiv((int)P, CB_BM), cdiv(H, 2) * a.ntw, B);
  hipLaunchKernelGGL(corr_build_kernel, grid, dim3(256), 0, s, a);
  int rc = check_launch("raft_corr_build");
  if (rc) return rc;
  size_t lvl_off[LK_MAXL];
  lvl_off[0] = 0;
  for (int l = 1; l < L; ++l) lvl_off[l] = lvl_off[l - 1] + (size_t)B * P * hs[l - 1] * ws[l - 1];
  for (int l = 2; l < L; ++l) {
    const long n = (long)B * P * hs[l] * ws[l];
    hipLaunchKernelGGL(pool2_kernel, dim3(grid_for(n)), dim3(256), 0, s, pyramid + lvl_off[l - 1],
                       pyramid + lvl_off[l], (long)B * P, hs[l - 1], ws[l - 1], hs[l], ws[l]);
    rc = check_launch("raft_corr_build(pool)");
    if (rc) return rc;
  }
  return 0;
}

extern "C" int raft_corr_lookup(const float* pyramid, int B, int H, int W, int L, int radius, const float* coords,
                                int coords_layout, float* out, int out_ld, int out_layout, float* flow_out,
                                int flow_ld, raft_stream_t stream) {
  RAFT_REQUIRE(pyramid && coords && out, "raft_corr_lookup: null pointer");
  RAFT_REQUIRE(B > 0 && H > 0 && W > 0 && L >= 1 && L <= LK_MAXL, "raft_corr_lookup: bad sizes");
  RAFT_REQUIRE(radius >= 1 && radius <= 4, "raft_corr_lookup: radius must be 1..4 (got %d)", radius);
  RAFT_REQUIRE(coords_layout == 0 || coords_layout == 1, "raft_corr_lookup: bad coords_layout");
  RAFT_REQUIRE(out_layout == 0 || out_layout == 1, "raft_corr_lookup: bad out_layout");
  const int rd = 2 * radius + 1;
  RAFT_REQUIRE(out_layout == 1 || out_ld >= L * rd * rd, "raft_corr_lookup: out_ld < L*(2r+1)^2");
  RAFT_REQUIRE(!flow_out || flow_ld >= 2, "raft_corr_lookup: flow_ld < 2");
  LookupArgs a;
  int hs[LK_MAXL], ws[LK_MAXL];
  pyramid_dims(H, W, L, hs, ws);
  const long P = (long)H * W;
  long off = 0;
  for (int l = 0; l < L; ++l) {
    RAFT_REQUIRE(hs[l] >= 1 && ws[l] >= 1, "raft_corr_lookup: level %d is empty", l);
    a.lvl_off[l] = off;
    a.lh[l] = hs[l];
    a.lw[l] = ws[l];
    off += (long)B * P * hs[l] * ws[l];
  }
  a.pyr = pyramid;
  a.B = B;
  a.H = H;
  a.W = W;
  a.L = L;
  a.r = radius;
  a.coords = coords;
  a.coords_layout = coords_layout;
  a.out = out;
  a.out_ld = out_ld;
  a.out_layout = out_layout;
  a.flow = flow_out;
  a.flow_ld = flow_ld;
  dim3 grid((unsigned)cdiv_l((long)B * P, 4));
  hipStream_t s = as_stream(stream);
  switch (radius) {
    case 1: hipLaunchKernelGGL(corr_lookup_kernel<1>, grid, dim3(256), 0, s, a); break;
    case 2: hipLaunchKernelGGL(corr_lookup_kernel<2>, grid, dim3(256), 0, s, a); break;
    case 3: hipLaunchKernelGGL(corr_lookup_kernel<3>, grid, dim3(256), 0, s, a); break;
    default: hipLaunchKernelGGL(corr_lookup_kernel<4>, grid, dim3(256), 0, s, a); break;
  }
  return check_launch("raft_corr_lookup");
}

static int alt_checks(const float* f1, const float* f2, const float* coords, const float* out, int B, int H1, int W1,
                      int H2, int W2, int C, int N, int r) {
  RAFT_REQUIRE(f1 && f2 && coords && out, "raft_alt_corr: null pointer");
  RAFT_REQUIRE(B > 0 && H1 > 0 && W1 > 0 && H2 > 0 && W2 > 0 && C > 0 && N > 0, "raft_alt_corr: bad sizes");
  RAFT_REQUIRE(C % 4 == 0 && C <= 1024, "raft_alt_corr: C must be a multiple of 4 and <= 1024 (got %d)", C);
  RAFT_REQUIRE(r >= 0 && (2 * r + 2) * (2 * r + 2) <= 128, "raft_alt_corr: radius must be 0..4 (got %d)", r);
  RAFT_REQUIRE((((uintptr_t)f1 | (uintptr_t)f2) & 15) == 0, "raft_alt_corr: fmaps must be 16-byte aligned");
  return 0;
}

extern "C" int raft_alt_corr_forward(const float* fmap1, const float* fmap2, const float* coords, float* corr, int B,
                                     int H1, int W1, int H2, int W2, int C, int N, int radius, float scale_div,
                                     raft_stream_t stream) {
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
  return launch_alt(a, stream);
}

extern "C" int raft_alt_corr_lookup_nhwc(const float* fmap1, const float* fmap2, const float* coords,
                                         int coords_layout, float coord_div, float* out, int out_ld, int B, int H1,
                                         int W1, int H2, int W2, int C, int radius, float scale_div, float* flow_out,
                                         int flow_ld, raft_stream_t stream) {
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
  return launch_alt(a, stream);
}

extern "C" size_t raft_alt_corr_backward_workspace_floats(int, int, int, int, int, int, int, int) { return 0; }

extern "C" int raft_alt_corr_backward(const float* fmap1, const float* fmap2, const float* coords,
                                      const float* corr_grad, float* fmap1_grad, float* fmap2_grad,
                                      float* coords_grad, int B, int H1, int W1, int H2, int W2, int C, int N,
                                      int radius, float*, size_t, raft_stream_t stream) {
  int rc = alt_checks(fmap1, fmap2, coords, corr_grad, B, H1, W1, H2, W2, C, N, radius);
  if (rc) return rc;
  RAFT_REQUIRE(fmap1_grad && fmap2_grad && coords_grad, "raft_alt_corr_backward: null gradient pointer");
  hipStream_t s = as_stream(stream);
  const long n2 = (long)B * H2 * W2 * C;
  const long nc = (long)B * N * H1 * W1 * 2;
  hipLaunchKernelGGL(zero_kernel, dim3(grid_for(n2)), dim3(256), 0, s, fmap2_grad, n2);
  hipLaunchKernelGGL(zero_kernel, dim3(grid_for(nc)), dim3(256), 0, s, coords_grad, nc);
  hipLaunchKernelGGL(alt_corr_bwd_kernel, dim3((unsigned)cdiv_l((long)B * H1 * W1, 4)), dim3(256), 0, s, fmap1,
                     fmap2, coords, corr_grad, fmap1_grad, fmap2_grad, B, H1, W1, H2, W2, C, N, radius);
  return check_launch("raft_alt_corr_backward");
}

extern "C" int raft_avgpool2_nhwc(const float* in, float* out, int B, int H, int W, int C, raft_stream_t stream) {
  RAFT_REQUIRE(in && out && B > 0 && H >= 2 && W >= 2 && C > 0, "raft_avgpool2_nhwc: bad arguments");
  const int Ho = H / 2, Wo = W / 2;
  const long n = (long)B * Ho * Wo * C;
  hipLaunchKernelGGL(avgpool2_nhwc_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), in, out, B, H, W, C,
                     Ho, Wo);
  return check_launch("raft_avgpool2_nhwc");
}
