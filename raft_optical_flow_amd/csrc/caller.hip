// Caller-side kernels of the RAFT inference path (gfx950): what demo.py / evaluate.py do
// around RAFT.forward, on the GPU instead of the host.
//
//   raft_pad_replicate        InputPadder.pad (core/utils/utils.py:7-24): replicate padding
//   raft_bilinear_sample      bilinear_sampler (core/utils/utils.py:57-71): grid_sample with
//                             align_corners=True and zero padding, in the reference's
//                             normalise / unnormalise arithmetic (as the lookup kernel)
//   raft_forward_interpolate  forward_interpolate (core/utils/utils.py:26-54): the Sintel
//                             warm start, scipy griddata(method='nearest') of the forward-
//                             splatted flow, as an exact fp64 nearest-neighbour search
#include "common.hpp"

namespace raft {
namespace {

__global__ void pad_replicate_kernel(const float* __restrict__ in, float* __restrict__ out, long nc, int H, int W,
                                     int top, int left, int Ho, int Wo) {
  const long total = nc * Ho * Wo;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = (int)(i % Wo);
    const long r = i / Wo;
    const int y = (int)(r % Ho);
    const long c = r / Ho;
    const int sy = min(max(y - top, 0), H - 1), sx = min(max(x - left, 0), W - 1);
    out[i] = in[(c * H + sy) * W + sx];
  }
}

// a / b correctly rounded from rcp = 1/b (rounded on the host): one Newton step
__device__ __forceinline__ float div_rn_(float a, float b, float rcp) {
  const float q = a * rcp;
  const float r = fmaf(-q, b, a);
  return fmaf(r, rcp, q);
}

// one axis of bilinear_sampler: pixel coordinate c -> 2c/(S-1) - 1 -> grid_sample's
// (g + 1) * ((S-1)/2); returns the floor and the fractional weight (NaN position -> !fin)
__device__ __forceinline__ bool sample_axis(float c, float m1, float rcp, int& i, float& t, float& g) {
  g = div_rn_(2.0f * c, m1, rcp) - 1.0f;
  const float u = (g + 1.0f) * (m1 * 0.5f);
  const bool fin = isfinite(u);
  const float f0 = fin ? floorf(u) : 0.f;
  t = u - f0;
  i = (int)f0;
  return fin;
}

__global__ void bilinear_sample_kernel(const float* __restrict__ img, const float* __restrict__ coords,
                                       float* __restrict__ out, float* __restrict__ mask, int N, int C, int H, int W,
                                       int Ho, int Wo, float wm1, float hm1, float rw, float rh) {
#pragma clang fp contract(off)  // the reference's bilinear is separate multiplies and adds
  const long P = (long)Ho * Wo;
  const long total = (long)N * P;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long n = i / P, p = i - n * P;
    const float x = coords[2 * i], y = coords[2 * i + 1];
    int ix, iy;
    float tx, ty, gx, gy;
    const bool fx = sample_axis(x, wm1, rw, ix, tx, gx);
    const bool fy = sample_axis(y, hm1, rh, iy, ty, gy);
    if (mask) mask[i] = (gx > -1.f && gy > -1.f && gx < 1.f && gy < 1.f) ? 1.f : 0.f;
    const bool in00 = (unsigned)ix < (unsigned)W && (unsigned)iy < (unsigned)H;
    const bool in01 = (unsigned)(ix + 1) < (unsigned)W && (unsigned)iy < (unsigned)H;
    const bool in10 = (unsigned)ix < (unsigned)W && (unsigned)(iy + 1) < (unsigned)H;
    const bool in11 = (unsigned)(ix + 1) < (unsigned)W && (unsigned)(iy + 1) < (unsigned)H;
    const float ex = 1.0f - tx, sS = 1.0f - ty;
    const float* base = img + n * C * (long)H * W;
    float* o = out + n * C * P + p;
    for (int c = 0; c < C; ++c) {
      const float* m = base + (long)c * H * W;
      const long r0 = (long)iy * W, r1 = r0 + W;
      const float v00 = in00 ? m[r0 + ix] : 0.f, v01 = in01 ? m[r0 + ix + 1] : 0.f;
      const float v10 = in10 ? m[r1 + ix] : 0.f, v11 = in11 ? m[r1 + ix + 1] : 0.f;
      const float v = v00 * (sS * ex) + v01 * (sS * tx) + v10 * (ty * ex) + v11 * (ty * tx);
      o[(long)c * P] = (fx && fy) ? v : __builtin_nanf("");
    }
  }
}

// Nearest valid forward-splatted source for every grid point of image b.  Source s = grid
// point (xs, ys) moved to (xs + dx, ys + dy) in fp64 (numpy's promotion of the float32 flow
// against the integer grid); valid when strictly inside (0, W) x (0, H).  Target (xt, yt)
// takes the flow of the source at the smallest squared distance, the lowest source index on
// a tie; no valid source -> 0 (griddata's fill_value).  256 targets per work-group, sources
// staged through LDS 256 at a time.
constexpr int FI_T = 256;
__global__ __launch_bounds__(FI_T) void forward_interpolate_kernel(const float* __restrict__ flow,
                                                                   float* __restrict__ out, int H, int W) {
  __shared__ double sx[FI_T], sy[FI_T];
  const int b = blockIdx.y;
  const int HW = H * W;
  const float* fx = flow + (long)b * 2 * HW;
  const float* fy = fx + HW;
  const int t = blockIdx.x * FI_T + threadIdx.x;
  const double xt = (double)(t % W), yt = (double)(t / W);
  double best = __builtin_inf();
  int bi = -1;
  for (int s0 = 0; s0 < HW; s0 += FI_T) {
    const int s = s0 + threadIdx.x;
    double x1 = __builtin_inf(), y1 = __builtin_inf();
    if (s < HW) {
      const double xa = (double)(s % W) + (double)fx[s], ya = (double)(s / W) + (double)fy[s];
      if (xa > 0.0 && xa < (double)W && ya > 0.0 && ya < (double)H) {
        x1 = xa;
        y1 = ya;
      }
    }
    __syncthreads();
    sx[threadIdx.x] = x1;
    sy[threadIdx.x] = y1;
    __syncthreads();
    const int n = min(FI_T, HW - s0);
    for (int k = 0; k < n; ++k) {
      const double ddx = sx[k] - xt, ddy = sy[k] - yt;
      const double d = ddx * ddx + ddy * ddy;  // inf for an invalid source: never taken
      if (d < best) {
        best = d;
        bi = s0 + k;
      }
    }
  }
  if (t < HW) {
    out[(long)b * 2 * HW + t] = bi >= 0 ? fx[bi] : 0.f;
    out[(long)b * 2 * HW + HW + t] = bi >= 0 ? fy[bi] : 0.f;
  }
}

int grid_1d(long n) {
  long g = (n + 255) / 256;
  return (int)(g > 65536 ? 65536 : g < 1 ? 1 : g);
}

}  // namespace
}  // namespace raft

using namespace raft;

extern "C" int raft_pad_replicate(const float* in, float* out, int NC, int H, int W, int top, int bottom, int left,
                                  int right, raft_stream_t stream) {
  RAFT_REQUIRE(in && out && NC > 0 && H > 0 && W > 0, "raft_pad_replicate: bad arguments");
  RAFT_REQUIRE(top >= 0 && bottom >= 0 && left >= 0 && right >= 0, "raft_pad_replicate: negative padding");
  const int Ho = H + top + bottom, Wo = W + left + right;
  hipLaunchKernelGGL(pad_replicate_kernel, dim3(grid_1d((long)NC * Ho * Wo)), dim3(256), 0, as_stream(stream), in,
                     out, (long)NC, H, W, top, left, Ho, Wo);
  return check_launch("raft_pad_replicate");
}

extern "C" int raft_bilinear_sample(const float* img, const float* coords, float* out, float* mask, int N, int C,
                                    int H, int W, int Ho, int Wo, raft_stream_t stream) {
  RAFT_REQUIRE(img && coords && out && N > 0 && C > 0 && H > 0 && W > 0 && Ho > 0 && Wo > 0,
               "raft_bilinear_sample: bad arguments");
  volatile float one = 1.0f;  // host IEEE division: the reciprocal the device refines
  const float wm1 = (float)(W - 1), hm1 = (float)(H - 1);
  hipLaunchKernelGGL(bilinear_sample_kernel, dim3(grid_1d((long)N * Ho * Wo)), dim3(256), 0, as_stream(stream), img,
                     coords, out, mask, N, C, H, W, Ho, Wo, wm1, hm1, one / wm1, one / hm1);
  return check_launch("raft_bilinear_sample");
}

extern "C" int raft_forward_interpolate(const float* flow, float* out, int B, int H, int W, raft_stream_t stream) {
  RAFT_REQUIRE(flow && out && B > 0 && H > 0 && W > 0 && B < 65536, "raft_forward_interpolate: bad arguments");
  RAFT_REQUIRE(flow != out, "raft_forward_interpolate: in-place is not supported");
  // the search is all-pairs (every target scans every source: (H W)^2 fp64 distances per image);
  // the RAFT warm start runs it at 1/8 resolution (Sintel: 55 x 128 = 7040 points, 5e7 pairs).
  // Beyond 2^16 points one launch would run for seconds (a GPU watchdog risk): refused.
  RAFT_REQUIRE((long)H * W <= RAFT_FI_MAX_POINTS,
               "raft_forward_interpolate: %d x %d = %ld points exceeds %d (the all-pairs nearest search is "
               "meant for 1/8-resolution flow)", H, W, (long)H * W, RAFT_FI_MAX_POINTS);
  dim3 grid((unsigned)cdiv_l((long)H * W, FI_T), (unsigned)B);
  hipLaunchKernelGGL(forward_interpolate_kernel, grid, dim3(FI_T), 0, as_stream(stream), flow, out, H, W);
  return check_launch("raft_forward_interpolate");
}
