// Backward of the alternate (on-the-fly) correlation: the alt_cuda_corr plugin's
// backward (alt_cuda_corr/correlation.cpp:36-48, correlation_kernel.cu:122-256,
// :288-324), for gfx950, deterministic and with the coordinate gradient.
//
// The forward (raft_alt_corr_forward) computes, per query q = (b, n, p) with
// x0 = floor(x) - r, y0 = floor(y) - r and tap t = (iy, ix) of the (2r+2)^2 window,
//   s_t = <fmap1[b, p], fmap2[b, y0 + iy, x0 + ix]>   (0 off the map)
//   corr[o = oy + (2r+1) ox] = s(oy,ox) (1-dy)(1-dx) + s(oy,ox+1) (1-dy) dx
//                            + s(oy+1,ox) dy (1-dx) + s(oy+1,ox+1) dy dx,
// dx = x - floor(x), dy = y - floor(y).  With G = corr_grad:
//   g_t            = sum of G over the (<= 4) bins tap t feeds, times their weights
//   fmap1_grad[b,p] = sum_n sum_t g_t fmap2[b, tap t]           (a gather: deterministic)
//   fmap2_grad[b,q2] = sum over every (query, tap) landing on q2 of g_t fmap1[b, p]
//   coords_grad     = sum_o G_o d corr_o / d(x, y)  (the weights' derivatives; the taps'
//                     floor is piecewise constant).  The reference leaves it zero (:307).
// The reference scatters fmap2_grad with float atomics (:237), so its low bits depend
// on the arrival order.  Here the (query, tap) -> fmap2 pixel map is inverted instead:
//   1. one wave per (b, p): tap sums, tap gradients g_t (kept in the workspace),
//      fmap1_grad, coords_grad, and the query's window-origin key (b, y0, x0);
//   2. a stable radix sort of the queries by that key (hipCUB, deterministic);
//   3. one wave per fmap2 pixel: the windows covering it have origins in a
//      (2r+2) x (2r+2) block of keys, i.e. 2r+2 contiguous key ranges of the sorted
//      list (two binary searches each); it sums g_t fmap1[p] over them in the sorted
//      order (key, then query index), which is fixed: bit-identical run to run.
#include <hipcub/hipcub.hpp>

#include "common.hpp"

namespace raft {
namespace {

constexpr int KEY_NONE = 0x7fffffff;  // a window that misses the map (or non-finite coords)

struct BwdArgs {
  const float *f1, *f2, *coords, *cg;
  float *f1g, *f2g, *crg;
  float* tapg;  // [Q][ntaps] tap gradients
  int* keys;    // [Q] window-origin keys (sort input)
  int* vals;    // [Q] query ids (sort input)
  const int* skeys;  // sorted
  const int* svals;
  int B, H1, W1, H2, W2, C, N, r;
  int ncell, cw;  // key cells per batch entry, cells per key row (W2 + wd - 1)
  long Q;
};

__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int m = 32; m >= 1; m >>= 1) v += __shfl_xor(v, m);
  return v;
}

// one wave per (b, p); loops over the N coordinate sets of the query pixel.  Dynamic LDS: per
// wave the (2r+2)^2 tap sums and tap gradients (any radius; blocks of 4 waves while that fits
// 64 KB, else of one wave: r <= 32 takes <= 35 KB per wave)
__global__ __launch_bounds__(256) void alt_bwd_query_kernel(BwdArgs a) {
  extern __shared__ float bwd_lds[];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, wpb = blockDim.x >> 6;
  const int P1 = a.H1 * a.W1;
  const long bp = (long)blockIdx.x * wpb + wv;
  if (bp >= (long)a.B * P1) return;
  const int b = (int)(bp / P1), p = (int)(bp - (long)b * P1);
  const int r = a.r, rd = 2 * r + 1, wd = 2 * r + 2, ntaps = wd * wd;
  const float* f1row = a.f1 + bp * a.C;
  const float* f2b = a.f2 + (long)b * a.H2 * a.W2 * a.C;
  float* s = bwd_lds + (long)wv * 2 * ntaps;
  float* gt = s + ntaps;
  // fmap1 gradient accumulators: lane owns channels 4*lane + 256*k
  constexpr int KMAX = 4;  // C <= 1024
  f32x4 acc[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  for (int n = 0; n < a.N; ++n) {
    const long q = ((long)b * a.N + n) * P1 + p;
    const float x = a.coords[2 * q], y = a.coords[2 * q + 1];
    const bool fin = isfinite(x) && isfinite(y) && fabsf(x) < 1e8f && fabsf(y) < 1e8f;
    const float fx = fin ? floorf(x) : 0.f, fy = fin ? floorf(y) : 0.f;
    const float dx = x - fx, dy = y - fy;
    const int x0 = (int)fx - r, y0 = (int)fy - r;
    // tap sums s_t
    for (int t = 0; t < ntaps; ++t) {
      const int h2 = y0 + t / wd, w2 = x0 + t % wd;
      float v = 0.f;
      if (fin && (unsigned)h2 < (unsigned)a.H2 && (unsigned)w2 < (unsigned)a.W2) {
        const float* row = f2b + ((long)h2 * a.W2 + w2) * a.C;
        for (int c = 4 * lane; c < a.C; c += 256) {
          const f32x4 u = *reinterpret_cast<const f32x4*>(row + c);
          const f32x4 f = *reinterpret_cast<const f32x4*>(f1row + c);
          v += f[0] * u[0] + f[1] * u[1] + f[2] * u[2] + f[3] * u[3];
        }
      }
      v = wave_sum(v);
      if (lane == 0) s[t] = v;
    }
    const float* G = a.cg + (((long)b * a.N + n) * rd * rd) * P1 + p;  // G[o * P1]
    // tap gradients g_t (lane t, t + 64)
    for (int t = lane; t < ntaps; t += 64) {
      const int iy = t / wd, ix = t % wd;
      float g = 0.f;
      if (fin) {
        if (iy > 0 && ix > 0) g += G[(long)((iy - 1) + rd * (ix - 1)) * P1] * (dy * dx);
        if (iy > 0 && ix < rd) g += G[(long)((iy - 1) + rd * ix) * P1] * (dy * (1.f - dx));
        if (iy < rd && ix > 0) g += G[(long)(iy + rd * (ix - 1)) * P1] * ((1.f - dy) * dx);
        if (iy < rd && ix < rd) g += G[(long)(iy + rd * ix) * P1] * ((1.f - dy) * (1.f - dx));
      }
      gt[t] = g;
      a.tapg[q * ntaps + t] = g;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    // coordinate gradient: sum_o G_o d corr_o / d(x, y)
    float gx = 0.f, gy = 0.f;
    for (int o = lane; o < rd * rd; o += 64) {
      const int ox = o / rd, oy = o % rd;
      const float go = fin ? G[(long)o * P1] : 0.f;
      const float s00 = s[oy * wd + ox], s01 = s[oy * wd + ox + 1];
      const float s10 = s[(oy + 1) * wd + ox], s11 = s[(oy + 1) * wd + ox + 1];
      gx += go * ((1.f - dy) * (s01 - s00) + dy * (s11 - s10));
      gy += go * ((1.f - dx) * (s10 - s00) + dx * (s11 - s01));
    }
    gx = wave_sum(gx);
    gy = wave_sum(gy);
    if (lane == 0) {
      a.crg[2 * q] = gx;
      a.crg[2 * q + 1] = gy;
    }
    // fmap1 gradient: sum_t g_t fmap2[tap t]
    for (int t = 0; t < ntaps; ++t) {
      const int h2 = y0 + t / wd, w2 = x0 + t % wd;
      if (!fin || (unsigned)h2 >= (unsigned)a.H2 || (unsigned)w2 >= (unsigned)a.W2) continue;
      const float g = gt[t];
      const float* row = f2b + ((long)h2 * a.W2 + w2) * a.C;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < a.C) acc[k] += g * *reinterpret_cast<const f32x4*>(row + c);
      }
    }
    // the window-origin key of this query (windows that miss the map sort last)
    if (lane == 0) {
      const bool hit = fin && x0 > -wd && x0 < a.W2 && y0 > -wd && y0 < a.H2;
      a.keys[q] = hit ? b * a.ncell + (y0 + wd - 1) * a.cw + (x0 + wd - 1) : KEY_NONE;
      a.vals[q] = (int)q;
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < a.C) *reinterpret_cast<f32x4*>(a.f1g + bp * a.C + c) = acc[k];
  }
}

// first index i in [0, n) with keys[i] >= key (keys sorted ascending)
__device__ __forceinline__ long lower_bound(const int* keys, long n, int key) {
  long lo = 0, hi = n;
  while (lo < hi) {
    const long mid = (lo + hi) >> 1;
    if (keys[mid] < key)
      lo = mid + 1;
    else
      hi = mid;
  }
  return lo;
}

// one wave per fmap2 pixel (b, h2, w2)
__global__ __launch_bounds__(256) void alt_bwd_fmap2_kernel(BwdArgs a) {
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const long P2 = (long)a.H2 * a.W2;
  const long gq = (long)blockIdx.x * 4 + wv;
  if (gq >= (long)a.B * P2) return;
  const int b = (int)(gq / P2);
  const int pq = (int)(gq - (long)b * P2);
  const int h2 = pq / a.W2, w2 = pq - h2 * a.W2;
  const int wd = 2 * a.r + 2, ntaps = wd * wd;
  const int P1 = a.H1 * a.W1;
  constexpr int KMAX = 4;
  f32x4 acc[KMAX];
#pragma unroll
  for (int k = 0; k < KMAX; ++k) acc[k] = f32x4{0.f, 0.f, 0.f, 0.f};
  // windows with origin (y0, x0), y0 in [h2 - wd + 1, h2], x0 in [w2 - wd + 1, w2], cover (h2, w2);
  // for one y0 their keys are contiguous
  for (int iy = wd - 1; iy >= 0; --iy) {
    const int y0 = h2 - iy;
    const int row = b * a.ncell + (y0 + wd - 1) * a.cw;
    const int klo = row + (w2 - (wd - 1) + wd - 1), khi = row + (w2 + wd - 1);
    const long j0 = __builtin_amdgcn_readfirstlane((int)lower_bound(a.skeys, a.Q, klo));
    const long j1 = __builtin_amdgcn_readfirstlane((int)lower_bound(a.skeys, a.Q, khi + 1));
    for (long j = j0; j < j1; ++j) {
      const int key = a.skeys[j];
      const int q = a.svals[j];
      const int x0 = (key - row) - (wd - 1);
      const int t = iy * wd + (w2 - x0);
      const float g = a.tapg[(long)q * ntaps + t];
      const int p = q % P1;
      const float* f1row = a.f1 + ((long)b * P1 + p) * a.C;
#pragma unroll
      for (int k = 0; k < KMAX; ++k) {
        const int c = 4 * lane + 256 * k;
        if (c < a.C) acc[k] += g * *reinterpret_cast<const f32x4*>(f1row + c);
      }
    }
  }
#pragma unroll
  for (int k = 0; k < KMAX; ++k) {
    const int c = 4 * lane + 256 * k;
    if (c < a.C) *reinterpret_cast<f32x4*>(a.f2g + gq * a.C + c) = acc[k];
  }
}

struct WsLayout {
  size_t sort_bytes, tapg_off, keys_off, vals_off, skeys_off, svals_off, total_bytes;
};

size_t align256(size_t v) { return (v + 255) & ~(size_t)255; }

int ws_layout(long Q, int ntaps, WsLayout& w) {
  size_t bytes = 0;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const int*)nullptr, (int*)nullptr,
                                                     (const int*)nullptr, (int*)nullptr, (int)Q, 0, 31);
  if (e != hipSuccess) return set_error((int)e, "raft_alt_corr_backward: sort size query failed");
  w.sort_bytes = align256(bytes);
  w.tapg_off = w.sort_bytes;
  w.keys_off = w.tapg_off + align256((size_t)Q * ntaps * 4);
  w.vals_off = w.keys_off + align256((size_t)Q * 4);
  w.skeys_off = w.vals_off + align256((size_t)Q * 4);
  w.svals_off = w.skeys_off + align256((size_t)Q * 4);
  w.total_bytes = w.svals_off + align256((size_t)Q * 4);
  return 0;
}

}  // namespace
}  // namespace raft

using namespace raft;

extern "C" size_t raft_alt_corr_backward_workspace_floats(int B, int H1, int W1, int H2, int W2, int C, int N,
                                                          int radius) {
  if (B <= 0 || H1 <= 0 || W1 <= 0 || H2 <= 0 || W2 <= 0 || C <= 0 || N <= 0 || radius < 0 || radius > 32) return 0;
  WsLayout w;
  if (ws_layout((long)B * N * H1 * W1, (2 * radius + 2) * (2 * radius + 2), w)) return 0;
  return (w.total_bytes + 3) / 4;
}

extern "C" int raft_alt_corr_backward(const float* fmap1, const float* fmap2, const float* coords,
                                      const float* corr_grad, float* fmap1_grad, float* fmap2_grad,
                                      float* coords_grad, int B, int H1, int W1, int H2, int W2, int C, int N,
                                      int radius, float* workspace, size_t workspace_floats, raft_stream_t stream) {
  RAFT_REQUIRE(fmap1 && fmap2 && coords && corr_grad, "raft_alt_corr_backward: null pointer");
  RAFT_REQUIRE(fmap1_grad && fmap2_grad && coords_grad, "raft_alt_corr_backward: null gradient pointer");
  RAFT_REQUIRE(B > 0 && H1 > 0 && W1 > 0 && H2 > 0 && W2 > 0 && N > 0, "raft_alt_corr_backward: bad sizes");
  RAFT_REQUIRE(C > 0 && C % 4 == 0 && C <= 1024, "raft_alt_corr_backward: C must be a multiple of 4, <= 1024");
  RAFT_REQUIRE(radius >= 0 && radius <= 32, "raft_alt_corr_backward: radius must be 0..32 (got %d)", radius);
  RAFT_REQUIRE(((((uintptr_t)fmap1) | ((uintptr_t)fmap2) | ((uintptr_t)fmap1_grad) | ((uintptr_t)fmap2_grad)) & 15) == 0,
               "raft_alt_corr_backward: fmaps and their gradients must be 16-byte aligned");
  const int wd = 2 * radius + 2;
  const long Q = (long)B * N * H1 * W1;
  const long cw = W2 + wd - 1, ncell = cw * (H2 + wd - 1);
  RAFT_REQUIRE(Q < (1L << 30) && (long)B * ncell < (long)KEY_NONE, "raft_alt_corr_backward: too large");
  WsLayout w;
  int rc = ws_layout(Q, wd * wd, w);
  if (rc) return rc;
  RAFT_REQUIRE(workspace && workspace_floats * 4 >= w.total_bytes,
               "raft_alt_corr_backward: workspace too small (raft_alt_corr_backward_workspace_floats)");
  char* ws = reinterpret_cast<char*>(workspace);
  BwdArgs a;
  a.f1 = fmap1;
  a.f2 = fmap2;
  a.coords = coords;
  a.cg = corr_grad;
  a.f1g = fmap1_grad;
  a.f2g = fmap2_grad;
  a.crg = coords_grad;
  a.tapg = reinterpret_cast<float*>(ws + w.tapg_off);
  a.keys = reinterpret_cast<int*>(ws + w.keys_off);
  a.vals = reinterpret_cast<int*>(ws + w.vals_off);
  a.skeys = reinterpret_cast<const int*>(ws + w.skeys_off);
  a.svals = reinterpret_cast<const int*>(ws + w.svals_off);
  a.B = B;
  a.H1 = H1;
  a.W1 = W1;
  a.H2 = H2;
  a.W2 = W2;
  a.C = C;
  a.N = N;
  a.r = radius;
  a.cw = (int)cw;
  a.ncell = (int)ncell;
  a.Q = Q;
  hipStream_t s = as_stream(stream);
  const size_t wave_lds = (size_t)2 * wd * wd * sizeof(float);
  const int wpb = 4 * wave_lds <= 65536 ? 4 : 1;
  hipLaunchKernelGGL(alt_bwd_query_kernel, dim3((unsigned)cdiv_l((long)B * H1 * W1, wpb)), dim3(64 * wpb),
                     wpb * wave_lds, s, a);
  rc = check_launch("raft_alt_corr_backward(query)");
  if (rc) return rc;
  size_t sb = w.sort_bytes;
  hipError_t e = hipcub::DeviceRadixSort::SortPairs(ws, sb, a.keys, const_cast<int*>(a.skeys), a.vals,
                                                     const_cast<int*>(a.svals), (int)Q, 0, 31, s);
  if (e != hipSuccess) return set_error((int)e, "raft_alt_corr_backward: sort failed: %s", hipGetErrorString(e));
  hipLaunchKernelGGL(alt_bwd_fmap2_kernel, dim3((unsigned)cdiv_l((long)B * H2 * W2, 4)), dim3(256), 0, s, a);
  return check_launch("raft_alt_corr_backward(fmap2)");
}
