// Elementwise / reduction kernels of the RAFT inference path (gfx950):
// image normalisation, InstanceNorm, coordinate state, convex upsampling.
#include "common.hpp"

namespace raft {

char* last_error_buf() {
  static thread_local char buf[512] = {0};
  return buf;
}

namespace {

int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

#define GRID_STRIDE(i, total) \
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < (total); i += (long)gridDim.x * blockDim.x)

// core/raft.py:164-169: 2 * (image / 255.0) - 1.0, NCHW -> NHWC, img1 batch then img2
__global__ void prep_images_kernel(const float* img1, const float* img2, float* out, int B, int H, int W) {
  const long HW = (long)H * W;
  const long total = 2L * B * HW * 3;
  GRID_STRIDE(i, total) {
    const int c = i % 3;
    const long pix = i / 3;  // (bb*H + y)*W + x
    const int bb = (int)(pix / HW);
    const long yx = pix - (long)bb * HW;
    const float* src = bb < B ? img1 + ((long)bb * 3 + c) * HW : img2 + ((long)(bb - B) * 3 + c) * HW;
    out[i] = 2.0f * (src[yx] / 255.0f) - 1.0f;
  }
}

// core/raft.py:89-110 + :208-209: coords1 = coords_grid (+ flow_init)
__global__ void init_coords_kernel(float* coords, const float* flow_init, int B, int H, int W) {
  const long P = (long)H * W;
  const long total = (long)B * P * 2;
  GRID_STRIDE(i, total) {
    const int c = i & 1;
    const long pix = i >> 1;
    const int b = (int)(pix / P);
    const long p = pix - (long)b * P;
    float v = c == 0 ? (float)(p % W) : (float)(p / W);
    if (flow_init) v = v + flow_init[((long)b * 2 + c) * P + p];
    coords[i] = v;
  }
}

// flow = coords1 - coords0, NCHW
__global__ void flow_from_coords_kernel(const float* coords, float* flow, int B, int H, int W) {
  const long P = (long)H * W;
  const long total = (long)B * 2 * P;
  GRID_STRIDE(i, total) {
    const long p = i % P;
    const long t = i / P;
    const int c = (int)(t % 2);
    const int b = (int)(t / 2);
    const float g = c == 0 ? (float)(p % W) : (float)(p / W);
    flow[i] = coords[((long)b * P + p) * 2 + c] - g;
  }
}

// RAFT.upsample_flow (core/raft.py:112-142).  One thread per output pixel
// (8h+a, 8w+b): softmax over the 9 mask logits k*64 + a*8 + b, weighted sum of
// 8*flow over the zero-padded 3x3 neighbourhood (k = ky*3 + kx).
__global__ void convex_upsample_kernel(const float* coords, const float* mask, int mask_ld, float* out, int B, int H,
                                       int W) {
  const int H8 = 8 * H, W8 = 8 * W;
  const long P8 = (long)H8 * W8;
  const long total = (long)B * P8;
  GRID_STRIDE(i, total) {
    const int X = i % W8;
    const long t = i / W8;
    const int Y = t % H8;
    const int b = (int)(t / H8);
    const int h = Y >> 3, a = Y & 7, w = X >> 3, bb = X & 7;
    const float* m = mask + ((long)b * H * W + (long)h * W + w) * mask_ld + a * 8 + bb;
    float lg[9];
    float mx = -INFINITY;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      lg[k] = m[k * 64];
      mx = fmaxf(mx, lg[k]);
    }
    float sum = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      lg[k] = expf(lg[k] - mx);
      sum += lg[k];
    }
    float fx = 0.f, fy = 0.f;
#pragma unroll
    for (int k = 0; k < 9; ++k) {
      const int yy = h + k / 3 - 1, xx = w + k % 3 - 1;
      float vx = 0.f, vy = 0.f;
      if (yy >= 0 && yy < H && xx >= 0 && xx < W) {
        const float* c = coords + ((long)b * H * W + (long)yy * W + xx) * 2;
        vx = 8.0f * (c[0] - (float)xx);
        vy = 8.0f * (c[1] - (float)yy);
      }
      const float wk = lg[k] / sum;
      fx += wk * vx;
      fy += wk * vy;
    }
    out[((long)b * 2) * P8 + (long)Y * W8 + X] = fx;
    out[((long)b * 2 + 1) * P8 + (long)Y * W8 + X] = fy;
  }
}

// upflow8 (core/utils/utils.py:80-82): 8 * bilinear(align_corners=True)
__global__ void upflow8_kernel(const float* coords, float* out, int B, int H, int W) {
  const int H8 = 8 * H, W8 = 8 * W;
  const long P8 = (long)H8 * W8;
  const float sy = H8 > 1 ? (float)(H - 1) / (float)(H8 - 1) : 0.f;
  const float sx = W8 > 1 ? (float)(W - 1) / (float)(W8 - 1) : 0.f;
  const long total = (long)B * 2 * P8;
  GRID_STRIDE(i, total) {
    const int X = i % W8;
    long t = i / W8;
    const int Y = t % H8;
    t /= H8;
    const int c = (int)(t % 2);
    const int b = (int)(t / 2);
    const float ry = sy * Y, rx = sx * X;
    const int y0 = min((int)ry, H - 1), x0 = min((int)rx, W - 1);
    const int y1 = y0 + (y0 < H - 1 ? 1 : 0), x1 = x0 + (x0 < W - 1 ? 1 : 0);
    const float ly = ry - y0, lx = rx - x0;
    auto f = [&](int yy, int xx) {
      return coords[((long)b * H * W + (long)yy * W + xx) * 2 + c] - (c == 0 ? (float)xx : (float)yy);
    };
    const float v = (1.f - ly) * ((1.f - lx) * f(y0, x0) + lx * f(y0, x1)) + ly * ((1.f - lx) * f(y1, x0) + lx * f(y1, x1));
    out[i] = 8.0f * v;
  }
}

__global__ void nchw_to_nhwc_kernel(const float* in, float* out, int ld, int B, int C, int H, int W) {
  const long P = (long)H * W;
  const long total = (long)B * P * C;
  GRID_STRIDE(i, total) {
    const int c = i % C;
    const long pix = i / C;
    const int b = (int)(pix / P);
    const long p = pix - (long)b * P;
    out[pix * ld + c] = in[((long)b * C + c) * P + p];
  }
}

__global__ void nhwc_to_nchw_kernel(const float* in, int ld, float* out, int B, int C, int H, int W) {
  const long P = (long)H * W;
  const long total = (long)B * C * P;
  GRID_STRIDE(i, total) {
    const long p = i % P;
    const long t = i / P;
    const int c = (int)(t % C);
    const int b = (int)(t / C);
    out[i] = in[((long)b * P + p) * ld + c];
  }
}

// InstanceNorm statistics, stage 1: per (image, pixel chunk) partial sums of
// (x - shift[c]) and (x - shift[c])^2 with shift = the image's first pixel
// (shifted data keeps E[x^2] - E[x]^2 well conditioned).
constexpr int IN_CHUNK = 256;  // pixels per partial-sum block: >= 2 blocks per CU at full res

__global__ __launch_bounds__(256) void instnorm_partial_kernel(const float* x, int ld, int HW, int C, float* part) {
  __shared__ float red[2][256];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int nchunk = gridDim.x;
  const int p0 = chunk * IN_CHUNK, p1 = min(HW, p0 + IN_CHUNK);
  const float* xb = x + (long)b * HW * ld;
  for (int cg = 0; cg < C; cg += 256) {
    const int ce = min(256, C - cg);
    const int R = 256 / ce;
    const int c = cg + threadIdx.x % ce, r = threadIdx.x / ce;
    float s = 0.f, ss = 0.f;
    if (r < R) {
      const float shift = xb[c];
      for (int p = p0 + r; p < p1; p += R) {
        const float d = xb[(long)p * ld + c] - shift;
        s += d;
        ss += d * d;
      }
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = ss;
    __syncthreads();
    if (threadIdx.x < ce) {
      float S = 0.f, SS = 0.f;
      for (int k = 0; k < R; ++k) {
        S += red[0][k * ce + threadIdx.x];
        SS += red[1][k * ce + threadIdx.x];
      }
      float* o = part + (((long)b * nchunk + chunk) * C + cg + threadIdx.x) * 2;
      o[0] = S;
      o[1] = SS;
    }
    __syncthreads();
  }
}

// Vectorised stage 1 (C and ld multiples of 4, x 16-B aligned): thread =
// (row r, channel quad q), 16-B loads, the same shifted sums per channel.
__global__ __launch_bounds__(256) void instnorm_partial4_kernel(const float* x, int ld, int HW, int C, float* part) {
  __shared__ f32x4 red[2][256];
  const int b = blockIdx.y, chunk = blockIdx.x;
  const int nchunk = gridDim.x;
  const int p0 = chunk * IN_CHUNK, p1 = min(HW, p0 + IN_CHUNK);
  const float* xb = x + (long)b * HW * ld;
  const int nq = C >> 2;
  for (int qg = 0; qg < nq; qg += 256) {
    const int qe = min(256, nq - qg);
    const int R = 256 / qe;
    const int q = qg + threadIdx.x % qe, r = threadIdx.x / qe;
    f32x4 s = {0.f, 0.f, 0.f, 0.f}, ss = s;
    if (r < R) {
      const f32x4 shift = *reinterpret_cast<const f32x4*>(xb + 4 * q);
#pragma unroll 4
      for (int p = p0 + r; p < p1; p += R) {
        const f32x4 d = *reinterpret_cast<const f32x4*>(xb + (long)p * ld + 4 * q) - shift;
        s += d;
        ss += d * d;
      }
    }
    red[0][threadIdx.x] = s;
    red[1][threadIdx.x] = ss;
    __syncthreads();
    if (threadIdx.x < qe) {
      f32x4 S = {0.f, 0.f, 0.f, 0.f}, SS = S;
      for (int k = 0; k < R; ++k) {
        S += red[0][k * qe + threadIdx.x];
        SS += red[1][k * qe + threadIdx.x];
      }
      f32x4* o = reinterpret_cast<f32x4*>(part + (((long)b * nchunk + chunk) * C + 4 * (qg + threadIdx.x)) * 2);
      o[0] = f32x4{S[0], SS[0], S[1], SS[1]};
      o[1] = f32x4{S[2], SS[2], S[3], SS[3]};
    }
    __syncthreads();
  }
}

// stage 2: one 256-thread block per (channel, image): thread t sums chunks t, t+256, ... in
// double, then a fixed-order LDS tree (deterministic).  One load round trip per thread
// instead of a 28-deep chain per thread of a 16-channel block (9 -> ~3 us at 1/2 res).
__global__ __launch_bounds__(256) void instnorm_finalize_kernel(const float* x, int ld, int HW, int C, int nchunk,
                                                                const float* part, float eps, float* stats, int B) {
  __shared__ double red[2][256];
  const int c = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  double S = 0.0, SS = 0.0;
  for (int k = t; k < nchunk; k += 256) {
    const float2 o = *reinterpret_cast<const float2*>(part + (((long)b * nchunk + k) * C + c) * 2);
    S += o.x;
    SS += o.y;
  }
  red[0][t] = S;
  red[1][t] = SS;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      red[0][t] += red[0][t + w];
      red[1][t] += red[1][t + w];
    }
    __syncthreads();
  }
  if (t != 0) return;
  S = red[0][0];
  SS = red[1][0];
  const int i = b * C + c;
  const double n = (double)HW;
  const double md = S / n;
  double var = SS / n - md * md;
  if (var < 0) var = 0;
  const double shift = x[(long)b * HW * ld + c];
  stats[2 * i] = (float)(shift + md);
  stats[2 * i + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

__global__ void instnorm_apply_kernel(const float* x, int ld, const float* stats, const float* resid, int rld,
                                      const float* rstats, int mode, float* out, int old, int B, int HW, int C) {
  const long total = (long)B * HW * C;
  GRID_STRIDE(i, total) {
    const int c = i % C;
    const long pix = i / C;
    const int b = (int)(pix / HW);
    const float* st = stats + 2 * ((long)b * C + c);
    float v = (x[pix * ld + c] - st[0]) * st[1];
    if (mode >= 1) v = fmaxf(v, 0.f);
    if (resid) {
      float r = resid[pix * rld + c];
      if (rstats) {
        const float* rs = rstats + 2 * ((long)b * C + c);
        r = (r - rs[0]) * rs[1];
      }
      v = r + v;
      if (mode == 2) v = fmaxf(v, 0.f);
    }
    out[pix * old + c] = v;
  }
}

// Vectorised apply (C, ld, resid_ld, out_ld multiples of 4, 16-B aligned rows):
// thread = (pixel, channel quad), 32-bit indexing (B*HW*C/4 < 2^31).
__global__ __launch_bounds__(256) void instnorm_apply4_kernel(const float* x, int ld, const float* stats,
                                                              const float* resid, int rld, const float* rstats, int mode,
                                                              float* out, int old, int HW, int nq, unsigned total) {
  for (unsigned i = blockIdx.x * 256u + threadIdx.x; i < total; i += gridDim.x * 256u) {
    const unsigned pix = i / (unsigned)nq, q = i - pix * (unsigned)nq;
    const unsigned b = pix / (unsigned)HW;
    const unsigned si = (b * (unsigned)nq + q) * 8u;  // (mean, rstd) of channels 4q .. 4q+3
    const f32x4 s0 = *reinterpret_cast<const f32x4*>(stats + si), s1 = *reinterpret_cast<const f32x4*>(stats + si + 4);
    const f32x4 xv = *reinterpret_cast<const f32x4*>(x + (size_t)pix * ld + 4 * q);
    f32x4 v = {(xv[0] - s0[0]) * s0[1], (xv[1] - s0[2]) * s0[3], (xv[2] - s1[0]) * s1[1], (xv[3] - s1[2]) * s1[3]};
    if (mode >= 1) {
#pragma unroll
      for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
    }
    if (resid) {
      f32x4 r = *reinterpret_cast<const f32x4*>(resid + (size_t)pix * rld + 4 * q);
      if (rstats) {
        const f32x4 r0 = *reinterpret_cast<const f32x4*>(rstats + si), r1 = *reinterpret_cast<const f32x4*>(rstats + si + 4);
        r = f32x4{(r[0] - r0[0]) * r0[1], (r[1] - r0[2]) * r0[3], (r[2] - r1[0]) * r1[1], (r[3] - r1[2]) * r1[3]};
      }
      v = r + v;
      if (mode == 2) {
#pragma unroll
        for (int e = 0; e < 4; ++e) v[e] = fmaxf(v[e], 0.f);
      }
    }
    *reinterpret_cast<f32x4*>(out + (size_t)pix * old + 4 * q) = v;
  }
}

// Chan's parallel merge of (count, mean, M2) partials, in double
__device__ __forceinline__ void chan_merge(double& n, double& mean, double& m2, double nb, double meanb, double m2b) {
  if (nb <= 0.0) return;
  const double nn = n + nb;
  const double d = meanb - mean;
  mean += d * (nb / nn);
  m2 += m2b + d * d * (n * nb / nn);
  n = nn;
}

// raft_instnorm_merge: one 256-thread block per (channel, image); thread t merges slots t, t+256, ...
// in order, then a fixed-order LDS tree (deterministic); stats = {mean, 1/sqrt(M2/n + eps)}
__global__ __launch_bounds__(256) void instnorm_merge_kernel(const float* part, int slots, int C, int ld, float eps,
                                                             float* stats) {
  __shared__ double red[3][256];
  const int c = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  double n = 0.0, mean = 0.0, m2 = 0.0;
  // 8 slots' loads in flight per thread, then their merges in slot order (the order, and so the
  // result, of one load-merge per slot; one memory latency per 8 slots instead of per slot)
  constexpr int PF = 8;
  for (int k0 = t; k0 < slots; k0 += 256 * PF) {
    f32x4 v[PF];
#pragma unroll
    for (int i = 0; i < PF; ++i) {
      const int k = k0 + 256 * i;
      v[i] = k < slots ? *reinterpret_cast<const f32x4*>(part + (((long)b * slots + k) * ld + c) * 4) : f32x4{};
    }
#pragma unroll
    for (int i = 0; i < PF; ++i)
      if (k0 + 256 * i < slots) chan_merge(n, mean, m2, (double)v[i][0], (double)v[i][1], (double)v[i][2]);
  }
  red[0][t] = n;
  red[1][t] = mean;
  red[2][t] = m2;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) {
      double n0 = red[0][t], m0 = red[1][t], q0 = red[2][t];
      chan_merge(n0, m0, q0, red[0][t + w], red[1][t + w], red[2][t + w]);
      red[0][t] = n0;
      red[1][t] = m0;
      red[2][t] = q0;
    }
    __syncthreads();
  }
  if (t != 0) return;
  const double nn = red[0][0];
  const double var = nn > 0.0 ? red[2][0] / nn : 0.0;
  stats[2 * (b * C + c)] = (float)red[1][0];
  stats[2 * (b * C + c) + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// raft_instnorm_merge_ws, level 1: block (channel group of 64, image, slot group g) sums its <= 64
// slots per channel relative to a shift K = the mean of slot 0 (sums only, no division: a fixed
// order, deterministic): n = sum c_i, s1 = sum c_i (m_i - K), s2 = sum M2_i + c_i (m_i - K)^2.
// Lane = channel (a wave's load of one slot is 1 KiB contiguous); wave w takes slots w, w+4, ...
constexpr int MERGE_SPG = 64;  // slots per level-1 group (4 waves x 16 loads in flight per lane)
__global__ __launch_bounds__(256) void instnorm_merge1_kernel(const float* part, int slots, int C, int ld,
                                                              double* ws, int G) {
  __shared__ double red[4][3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, b = blockIdx.y, g = blockIdx.z;
  const bool cok = c < C;
  const float* pb = part + ((long)b * slots * ld + (cok ? c : 0)) * 4;
  const float K = cok ? pb[1] : 0.f;  // slot 0's mean (slot 0 always holds pixels)
  f32x4 v[MERGE_SPG / 4];
#pragma unroll
  for (int i = 0; i < MERGE_SPG / 4; ++i) {
    const int k = g * MERGE_SPG + w + 4 * i;
    v[i] = (cok && k < slots) ? *reinterpret_cast<const f32x4*>(pb + (long)k * ld * 4) : f32x4{};
  }
  double n = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int i = 0; i < MERGE_SPG / 4; ++i) {
    const double cnt = v[i][0], d = (double)v[i][1] - (double)K;
    n += cnt;
    s1 += cnt * d;
    s2 += (double)v[i][2] + cnt * d * d;
  }
  red[w][0][lane] = n;
  red[w][1][lane] = s1;
  red[w][2][lane] = s2;
  __syncthreads();
  if (w == 0 && cok) {
    double* o = ws + (((long)b * G + g) * C + c) * 3;
#pragma unroll
    for (int q = 0; q < 3; ++q) o[q] = ((red[0][q][lane] + red[1][q][lane]) + red[2][q][lane]) + red[3][q][lane];
  }
}
// level 2: block (channel group of 64, image), 16 waves: wave w sums groups w, w + 16, ... (8 loads
// in flight per lane: one memory round trip per 128 groups), then wave 0 adds the 16 wave sums in
// order (deterministic) and writes {mean, rstd}
constexpr int MERGE2_WAVES = 16;
__global__ __launch_bounds__(64 * MERGE2_WAVES) void instnorm_merge2_kernel(const float* part, int slots, int C,
                                                                           int ld, const double* ws, int G, float eps,
                                                                           float* stats) {
  __shared__ double red[MERGE2_WAVES][3][64];
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, b = blockIdx.y;
  const bool cok = c < C;
  double n = 0.0, s1 = 0.0, s2 = 0.0;
  const double* p = ws + ((long)b * G * C + (cok ? c : 0)) * 3;
  for (int g0 = w; g0 < G; g0 += 8 * MERGE2_WAVES) {
    double t[8][3];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int g = g0 + MERGE2_WAVES * i;
#pragma unroll
      for (int q = 0; q < 3; ++q) t[i][q] = (cok && g < G) ? p[((long)g * C) * 3 + q] : 0.0;
    }
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      n += t[i][0];
      s1 += t[i][1];
      s2 += t[i][2];
    }
  }
  red[w][0][lane] = n;
  red[w][1][lane] = s1;
  red[w][2][lane] = s2;
  __syncthreads();
  if (w != 0 || !cok) return;
  n = s1 = s2 = 0.0;
#pragma unroll
  for (int k = 0; k < MERGE2_WAVES; ++k) {
    n += red[k][0][lane];
    s1 += red[k][1][lane];
    s2 += red[k][2][lane];
  }
  const double K = part[((long)b * slots * ld + c) * 4 + 1];
  const double mean = n > 0.0 ? K + s1 / n : 0.0;
  const double m2 = n > 0.0 ? fmax(s2 - s1 * s1 / n, 0.0) : 0.0;
  const double var = n > 0.0 ? m2 / n : 0.0;
  stats[2 * ((long)b * C + c)] = (float)mean;
  stats[2 * ((long)b * C + c) + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// raft_instnorm_merge_fused: level 1 and level 2 in ONE launch.  Each level-1 block stores its
// group's sums write-through (sc1) and adds to the (channel group, image) counter; the block whose add
// comes last runs level 2 over the G group sums (sc1 loads, after its add returned / a block barrier:
// MI355X_MICROARCH.md's last-arriver hand-off) in exactly merge2's order, so the statistics equal
// raft_instnorm_merge_ws's bit for bit; it then clears the counter for the next launch.
__global__ __launch_bounds__(64 * MERGE2_WAVES) void instnorm_merge_fused_kernel(const float* part, int slots, int C, int ld,
                                                                   double* ws, int G, float eps, float* stats,
                                                                   int* counters) {
  __shared__ double red[MERGE2_WAVES][3][64];  // (level 1 uses rows 0-3)
  __shared__ int is_last;
  const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lane, b = blockIdx.y, g = blockIdx.z;
  const bool cok = c < C;
  const float* pb = part + ((long)b * slots * ld + (cok ? c : 0)) * 4;
  const float K = cok ? pb[1] : 0.f;  // slot 0's mean (slot 0 always holds pixels)
  // (1024 threads: waves 0-3 run level 1 exactly as instnorm_merge1_kernel, all 16 waves level 2
  // exactly as instnorm_merge2_kernel, so the last block's tail is as parallel as that launch)
  if (w < 4) {
    f32x4 v[MERGE_SPG / 4];
#pragma unroll
    for (int i = 0; i < MERGE_SPG / 4; ++i) {
      const int k = g * MERGE_SPG + w + 4 * i;
      v[i] = (cok && k < slots) ? *reinterpret_cast<const f32x4*>(pb + (long)k * ld * 4) : f32x4{};
    }
    double n = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
    for (int i = 0; i < MERGE_SPG / 4; ++i) {
      const double cnt = v[i][0], d = (double)v[i][1] - (double)K;
      n += cnt;
      s1 += cnt * d;
      s2 += (double)v[i][2] + cnt * d * d;
    }
    red[w][0][lane] = n;
    red[w][1][lane] = s1;
    red[w][2][lane] = s2;
  }
  __syncthreads();
  int* cnt = counters + (long)b * gridDim.x + blockIdx.x;
  if (w == 0) {
    if (cok) {
      unsigned long long* o = reinterpret_cast<unsigned long long*>(ws + (((long)b * G + g) * C + c) * 3);
#pragma unroll
      for (int q = 0; q < 3; ++q)
        __hip_atomic_store(o + q,
                           __double_as_longlong(((red[0][q][lane] + red[1][q][lane]) + red[2][q][lane]) + red[3][q][lane]),
                           __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    // the sums have left for memory (sc1).  The hand-off is the measured valid form of
    // MI355X_MICROARCH.md (inter-workgroup visibility, first row of the sc1 table): every byte stored
    // sc1 and drained before ONE lane's agent-scope add; the block whose add returns G - 1 reads them
    // with sc1 loads only, behind a workgroup barrier, so no L1-resident copy can be read stale.  An
    // acq_rel add would order the same bytes through a whole-L2 write-back and an L1 invalidate
    // (~1.7 us each on this chip) per merge.
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (lane == 0) is_last = __hip_atomic_fetch_add(cnt, 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == G - 1;
  }
  __syncthreads();
  if (!is_last) return;
  // level 2 (merge2's order: wave k sums groups k, k + 16, ... in batches of 8)
  const unsigned long long* p = reinterpret_cast<const unsigned long long*>(ws + ((long)b * G * C + (cok ? c : 0)) * 3);
  {
    const int kk = w;
    double n = 0.0, s1 = 0.0, s2 = 0.0;
    for (int g0 = kk; g0 < G; g0 += 8 * MERGE2_WAVES) {
      double t[8][3];
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        const int gg = g0 + MERGE2_WAVES * i;
#pragma unroll
        for (int q = 0; q < 3; ++q)
          t[i][q] = (cok && gg < G) ? __longlong_as_double(__hip_atomic_load(p + (long)gg * C * 3 + q, __ATOMIC_RELAXED,
                                                                              __HIP_MEMORY_SCOPE_AGENT))
                                    : 0.0;
      }
#pragma unroll
      for (int i = 0; i < 8; ++i) {
        n += t[i][0];
        s1 += t[i][1];
        s2 += t[i][2];
      }
    }
    red[kk][0][lane] = n;
    red[kk][1][lane] = s1;
    red[kk][2][lane] = s2;
  }
  __syncthreads();
  if (w != 0) return;
  // the next launch starts from zero (an agent-scope store, like every other access to the counter; the
  // kernel boundary orders it before the next launch's adds)
  if (lane == 0) __hip_atomic_store(cnt, 0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  if (!cok) return;
  double n = 0.0, s1 = 0.0, s2 = 0.0;
#pragma unroll
  for (int k = 0; k < MERGE2_WAVES; ++k) {
    n += red[k][0][lane];
    s1 += red[k][1][lane];
    s2 += red[k][2][lane];
  }
  const double Kd = K;
  const double mean = n > 0.0 ? Kd + s1 / n : 0.0;
  const double m2 = n > 0.0 ? fmax(s2 - s1 * s1 / n, 0.0) : 0.0;
  const double var = n > 0.0 ? m2 / n : 0.0;
  stats[2 * ((long)b * C + c)] = (float)mean;
  stats[2 * ((long)b * C + c) + 1] = (float)(1.0 / sqrt(var + (double)eps));
}

// nn.GroupNorm statistics (core/extractor.py:23-25, the blocks' norm_fn='group'): one block per
// (group, image); mean, then the variance around it, over the group's C/G channels x HW pixels in
// double with a fixed-order tree (deterministic); written per (image, channel) as the {mean, rstd}
// of the channel's group.
__device__ double block_sum256(double v, double* red) {
  const int t = threadIdx.x;
  red[t] = v;
  __syncthreads();
  for (int w = 128; w > 0; w >>= 1) {
    if (t < w) red[t] += red[t + w];
    __syncthreads();
  }
  const double r = red[0];
  __syncthreads();
  return r;
}
__global__ __launch_bounds__(256) void groupnorm_stats_kernel(const float* x, int ld, int HW, int C, int G, float eps,
                                                              float* stats) {
  __shared__ double red[256];
  const int g = blockIdx.x, b = blockIdx.y, t = threadIdx.x;
  const int cg = C / G, c0 = g * cg;
  const long n = (long)HW * cg;
  const float* xb = x + (long)b * HW * ld + c0;
  double s = 0.0;
  for (long i = t; i < n; i += 256) {
    const long pix = i / cg;
    s += (double)xb[pix * ld + (i - pix * cg)];
  }
  const double mean = block_sum256(s, red) / (double)n;
  double q = 0.0;
  for (long i = t; i < n; i += 256) {
    const long pix = i / cg;
    const double d = (double)xb[pix * ld + (i - pix * cg)] - mean;
    q += d * d;
  }
  const double var = block_sum256(q, red) / (double)n;
  for (int c = t; c < cg; c += 256) {
    stats[2 * ((long)b * C + c0 + c)] = (float)mean;
    stats[2 * ((long)b * C + c0 + c) + 1] = (float)(1.0 / sqrt(var + (double)eps));
  }
}

// The normalisation with a per-channel affine (GroupNorm's weight / bias): v = (x - mean) * rstd *
// gamma[c] + beta[c], relu (mode >= 1), + the residual (itself normalised and scaled when rstats /
// rgamma / rbeta are given), relu (mode 2): raft_instnorm_apply plus the affine.
__global__ void norm_apply_affine_kernel(const float* x, int ld, const float* stats, const float* gamma,
                                         const float* beta, const float* resid, int rld, const float* rstats,
                                         const float* rgamma, const float* rbeta, int mode, float* out, int old, int B,
                                         int HW, int C) {
  const long total = (long)B * HW * C;
  GRID_STRIDE(i, total) {
    const int c = i % C;
    const long pix = i / C;
    const int b = (int)(pix / HW);
    const float* st = stats + 2 * ((long)b * C + c);
    float v = (x[pix * ld + c] - st[0]) * st[1];
    if (gamma) v = v * gamma[c];
    if (beta) v = v + beta[c];
    if (mode >= 1) v = fmaxf(v, 0.f);
    if (resid) {
      float r = resid[pix * rld + c];
      if (rstats) {
        const float* rs = rstats + 2 * ((long)b * C + c);
        r = (r - rs[0]) * rs[1];
        if (rgamma) r = r * rgamma[c];
        if (rbeta) r = r + rbeta[c];
      }
      v = r + v;
      if (mode == 2) v = fmaxf(v, 0.f);
    }
    out[pix * old + c] = v;
  }
}

bool aligned16(const void* q) { return ((uintptr_t)q & 15) == 0; }

// Debug: every work-group takes a CU's whole LDS (160 KiB) and fills it with all-ones words (a NaN
// as one fp32 or two f16 / bf16 values), so the next kernel on that CU starts with NaN wherever it
// reads LDS it did not write.  Only the value of LDS changes: no global memory is touched.
constexpr int LDS_FILL_BYTES = 160 * 1024;
__global__ __launch_bounds__(1024) void fill_lds_nan_kernel() {
  extern __shared__ __attribute__((aligned(16))) unsigned lds_fill[];
  const unsigned ones = 0xffffffffu;
  for (int i = threadIdx.x; i < LDS_FILL_BYTES / 16; i += blockDim.x)
    reinterpret_cast<uint4*>(lds_fill)[i] = make_uint4(ones, ones, ones, ones);
  __syncthreads();
}

}  // namespace
}  // namespace raft

using namespace raft;

extern "C" int raft_hip_abi_version(void) { return RAFT_HIP_ABI_VERSION; }

#ifndef RAFT_SRC_HASH
#define RAFT_SRC_HASH "unknown"
#endif
extern "C" const char* raft_hip_source_hash(void) { return RAFT_SRC_HASH; }
extern "C" const char* raft_hip_arch(void) { return "gfx950"; }
extern "C" const char* raft_hip_last_error(void) { return last_error_buf(); }

extern "C" int raft_prep_images(const float* img1, const float* img2, float* out, int B, int H, int W,
                                raft_stream_t stream) {
  RAFT_REQUIRE(img1 && img2 && out && B > 0 && H > 0 && W > 0, "raft_prep_images: bad arguments");
  const long n = 2L * B * H * W * 3;
  hipLaunchKernelGGL(prep_images_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), img1, img2, out, B, H,
                     W);
  return check_launch("raft_prep_images");
}

extern "C" int raft_init_coords(float* coords, const float* flow_init, int B, int H, int W, raft_stream_t stream) {
  RAFT_REQUIRE(coords && B > 0 && H > 0 && W > 0, "raft_init_coords: bad arguments");
  const long n = (long)B * H * W * 2;
  hipLaunchKernelGGL(init_coords_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), coords, flow_init, B, H,
                     W);
  return check_launch("raft_init_coords");
}

extern "C" int raft_flow_from_coords(const float* coords, float* flow, int B, int H, int W, raft_stream_t stream) {
  RAFT_REQUIRE(coords && flow && B > 0 && H > 0 && W > 0, "raft_flow_from_coords: bad arguments");
  const long n = (long)B * H * W * 2;
  hipLaunchKernelGGL(flow_from_coords_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), coords, flow, B, H,
                     W);
  return check_launch("raft_flow_from_coords");
}

extern "C" int raft_convex_upsample(const float* coords, const float* mask, int mask_ld, float* flow_up, int B, int H,
                                    int W, raft_stream_t stream) {
  RAFT_REQUIRE(coords && mask && flow_up && B > 0 && H > 0 && W > 0, "raft_convex_upsample: bad arguments");
  RAFT_REQUIRE(mask_ld >= 576, "raft_convex_upsample: mask_ld must be >= 576");
  const long n = (long)B * 64 * H * W;
  hipLaunchKernelGGL(convex_upsample_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), coords, mask,
                     mask_ld, flow_up, B, H, W);
  return check_launch("raft_convex_upsample");
}

extern "C" int raft_upflow8(const float* coords, float* flow_up, int B, int H, int W, raft_stream_t stream) {
  RAFT_REQUIRE(coords && flow_up && B > 0 && H > 0 && W > 0, "raft_upflow8: bad arguments");
  const long n = (long)B * 2 * 64 * H * W;
  hipLaunchKernelGGL(upflow8_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), coords, flow_up, B, H, W);
  return check_launch("raft_upflow8");
}

extern "C" int raft_nchw_to_nhwc(const float* in, float* out, int out_ld, int B, int C, int H, int W,
                                 raft_stream_t stream) {
  RAFT_REQUIRE(in && out && B > 0 && C > 0 && H > 0 && W > 0 && out_ld >= C, "raft_nchw_to_nhwc: bad arguments");
  const long n = (long)B * C * H * W;
  hipLaunchKernelGGL(nchw_to_nhwc_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), in, out, out_ld, B, C,
                     H, W);
  return check_launch("raft_nchw_to_nhwc");
}

extern "C" int raft_nhwc_to_nchw(const float* in, int in_ld, float* out, int B, int C, int H, int W,
                                 raft_stream_t stream) {
  RAFT_REQUIRE(in && out && B > 0 && C > 0 && H > 0 && W > 0 && in_ld >= C, "raft_nhwc_to_nchw: bad arguments");
  const long n = (long)B * C * H * W;
  hipLaunchKernelGGL(nhwc_to_nchw_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), in, in_ld, out, B, C,
                     H, W);
  return check_launch("raft_nhwc_to_nchw");
}

extern "C" size_t raft_instnorm_workspace_floats(int B, int HW, int C) {
  if (B <= 0 || HW <= 0 || C <= 0) return 0;
  const long nchunk = cdiv_l(HW, IN_CHUNK);
  return (size_t)B * nchunk * C * 2;
}

extern "C" int raft_instnorm_stats(const float* x, int ld, int B, int HW, int C, float eps, float* stats,
                                   float* workspace, raft_stream_t stream) {
  RAFT_REQUIRE(x && stats && workspace && B > 0 && HW > 0 && C > 0 && ld >= C, "raft_instnorm_stats: bad arguments");
  const int nchunk = (int)cdiv_l(HW, IN_CHUNK);
  hipStream_t s = as_stream(stream);
  if (C % 4 == 0 && ld % 4 == 0 && aligned16(x) && aligned16(workspace))
    hipLaunchKernelGGL(instnorm_partial4_kernel, dim3(nchunk, B), dim3(256), 0, s, x, ld, HW, C, workspace);
  else
    hipLaunchKernelGGL(instnorm_partial_kernel, dim3(nchunk, B), dim3(256), 0, s, x, ld, HW, C, workspace);
  int rc = check_launch("raft_instnorm_stats(partial)");
  if (rc) return rc;
  hipLaunchKernelGGL(instnorm_finalize_kernel, dim3(C, B), dim3(256), 0, s, x, ld, HW, C, nchunk, workspace, eps,
                     stats, B);
  return check_launch("raft_instnorm_stats(finalize)");
}

extern "C" int raft_instnorm_merge(const float* part, int slots_per_image, int B, int C, int stats_ld, float eps,
                                   float* stats, raft_stream_t stream) {
  RAFT_REQUIRE(part && stats && slots_per_image > 0 && B > 0 && C > 0 && stats_ld >= C && B < 65536,
               "raft_instnorm_merge: bad arguments");
  RAFT_REQUIRE(aligned16(part), "raft_instnorm_merge: part must be 16-byte aligned");
  hipLaunchKernelGGL(instnorm_merge_kernel, dim3(C, B), dim3(256), 0, as_stream(stream), part, slots_per_image, C,
                     stats_ld, eps, stats);
  return check_launch("raft_instnorm_merge");
}

extern "C" size_t raft_instnorm_merge_ws_floats(int slots_per_image, int B, int C) {
  if (slots_per_image <= 0 || B <= 0 || C <= 0) return 0;
  return (size_t)B * cdiv(slots_per_image, MERGE_SPG) * C * 3 * 2;  // doubles
}

extern "C" int raft_instnorm_merge_ws(const float* part, int slots_per_image, int B, int C, int stats_ld, float eps,
                                      void* ws, float* stats, raft_stream_t stream) {
  RAFT_REQUIRE(part && ws && stats && slots_per_image > 0 && B > 0 && C > 0 && stats_ld >= C && B < 65536,
               "raft_instnorm_merge_ws: bad arguments");
  RAFT_REQUIRE(aligned16(part) && ((uintptr_t)ws & 7) == 0, "raft_instnorm_merge_ws: part 16-B, ws 8-B aligned");
  const int G = cdiv(slots_per_image, MERGE_SPG);
  RAFT_REQUIRE(G < 65536, "raft_instnorm_merge_ws: too many slots");
  hipStream_t s = as_stream(stream);
  hipLaunchKernelGGL(instnorm_merge1_kernel, dim3(cdiv(C, 64), B, G), dim3(256), 0, s, part, slots_per_image, C,
                     stats_ld, reinterpret_cast<double*>(ws), G);
  hipLaunchKernelGGL(instnorm_merge2_kernel, dim3(cdiv(C, 64), B), dim3(64 * MERGE2_WAVES), 0, s, part, slots_per_image, C, stats_ld,
                     reinterpret_cast<const double*>(ws), G, eps, stats);
  return check_launch("raft_instnorm_merge_ws");
}

extern "C" size_t raft_instnorm_merge_counters(int B, int C) {
  if (B <= 0 || C <= 0) return 0;
  return (size_t)B * cdiv(C, 64);
}

extern "C" int raft_instnorm_merge_fused(const float* part, int slots_per_image, int B, int C, int stats_ld, float eps,
                                         void* ws, int* counters, float* stats, raft_stream_t stream) {
  RAFT_REQUIRE(part && ws && counters && stats && slots_per_image > 0 && B > 0 && C > 0 && stats_ld >= C && B < 65536,
               "raft_instnorm_merge_fused: bad arguments");
  RAFT_REQUIRE(aligned16(part) && ((uintptr_t)ws & 7) == 0 && ((uintptr_t)counters & 3) == 0,
               "raft_instnorm_merge_fused: part 16-B, ws 8-B, counters 4-B aligned");
  const int G = cdiv(slots_per_image, MERGE_SPG);
  RAFT_REQUIRE(G < 65536, "raft_instnorm_merge_fused: too many slots");
  hipLaunchKernelGGL(instnorm_merge_fused_kernel, dim3(cdiv(C, 64), B, G), dim3(64 * MERGE2_WAVES), 0, as_stream(stream), part,
                     slots_per_image, C, stats_ld, reinterpret_cast<double*>(ws), G, eps, stats, counters);
  return check_launch("raft_instnorm_merge_fused");
}

extern "C" int raft_instnorm_apply(const float* x, int ld, const float* stats, const float* resid, int resid_ld,
                                   const float* resid_stats, int relu_mode, float* out, int out_ld, int B, int HW,
                                   int C, raft_stream_t stream) {
  RAFT_REQUIRE(x && stats && out && B > 0 && HW > 0 && C > 0 && ld >= C && out_ld >= C,
               "raft_instnorm_apply: bad arguments");
  RAFT_REQUIRE(relu_mode >= 0 && relu_mode <= 2, "raft_instnorm_apply: bad relu_mode");
  RAFT_REQUIRE(!resid || resid_ld >= C, "raft_instnorm_apply: bad resid_ld");
  const long n = (long)B * HW * C;
  const bool vec = C % 4 == 0 && ld % 4 == 0 && out_ld % 4 == 0 && aligned16(x) && aligned16(out) &&
                   aligned16(stats) && (!resid || (resid_ld % 4 == 0 && aligned16(resid))) &&
                   (!resid_stats || aligned16(resid_stats)) && n / 4 < (1L << 31);
  if (vec)
    hipLaunchKernelGGL(instnorm_apply4_kernel, dim3(grid_for(n / 4)), dim3(256), 0, as_stream(stream), x, ld, stats,
                       resid, resid_ld, resid_stats, relu_mode, out, out_ld, HW, C / 4, (unsigned)(n / 4));
  else
    hipLaunchKernelGGL(instnorm_apply_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, ld, stats, resid,
                       resid_ld, resid_stats, relu_mode, out, out_ld, B, HW, C);
  return check_launch("raft_instnorm_apply");
}

extern "C" int raft_groupnorm_stats(const float* x, int ld, int B, int HW, int C, int G, float eps, float* stats,
                                    raft_stream_t stream) {
  RAFT_REQUIRE(x && stats && B > 0 && HW > 0 && C > 0 && G > 0 && C % G == 0 && ld >= C && B < 65536 && G < 65536,
               "raft_groupnorm_stats: bad arguments (C %% G == 0 required)");
  hipLaunchKernelGGL(groupnorm_stats_kernel, dim3(G, B), dim3(256), 0, as_stream(stream), x, ld, HW, C, G, eps, stats);
  return check_launch("raft_groupnorm_stats");
}

extern "C" int raft_norm_apply_affine(const float* x, int ld, const float* stats, const float* gamma, const float* beta,
                                      const float* resid, int resid_ld, const float* resid_stats,
                                      const float* resid_gamma, const float* resid_beta, int relu_mode, float* out,
                                      int out_ld, int B, int HW, int C, raft_stream_t stream) {
  RAFT_REQUIRE(x && stats && out && B > 0 && HW > 0 && C > 0 && ld >= C && out_ld >= C,
               "raft_norm_apply_affine: bad arguments");
  RAFT_REQUIRE(relu_mode >= 0 && relu_mode <= 2, "raft_norm_apply_affine: bad relu_mode");
  RAFT_REQUIRE(!resid || resid_ld >= C, "raft_norm_apply_affine: bad resid_ld");
  const long n = (long)B * HW * C;
  hipLaunchKernelGGL(norm_apply_affine_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), x, ld, stats, gamma,
                     beta, resid, resid_ld, resid_stats, resid_gamma, resid_beta, relu_mode, out, out_ld, B, HW, C);
  return check_launch("raft_norm_apply_affine");
}

extern "C" int raft_debug_fill_lds_nan(raft_stream_t stream) {
  int dev = 0, cus = 0;
  RAFT_REQUIRE(hipGetDevice(&dev) == hipSuccess &&
               hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && cus > 0,
               "raft_debug_fill_lds_nan: no device");
  static bool attr = [] {
    return hipFuncSetAttribute(reinterpret_cast<const void*>(fill_lds_nan_kernel),
                               hipFuncAttributeMaxDynamicSharedMemorySize, LDS_FILL_BYTES) == hipSuccess;
  }();
  RAFT_REQUIRE(attr, "raft_debug_fill_lds_nan: cannot request %d B of LDS", LDS_FILL_BYTES);
  // several work-groups per CU, one resident at a time (the LDS), so every CU runs at least one
  hipLaunchKernelGGL(fill_lds_nan_kernel, dim3((unsigned)(4 * cus)), dim3(1024), LDS_FILL_BYTES, as_stream(stream));
  return check_launch("raft_debug_fill_lds_nan");
}
