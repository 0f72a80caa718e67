// Implicit-GEMM convolution on fp32 MFMA (v_mfma_f32_32x32x2_f32) for gfx950.
//
// Replaces every nn.Conv2d of the RAFT update block (core/update.py:6-325) and
// encoders (core/extractor.py:6-267), with the surrounding elementwise work of
// the reference fused into the epilogue (ReLU, residual add, GRU gates and
// blend, tanh/relu split of the context net, coords1 += delta_flow).
//
// Layout: NHWC rows.  GEMM view: M = output pixels, N = output channels,
// K = (tap, channel).  Work-group tile 64(M) x 64(N), K-step 32; four waves in
// a 2x2 arrangement each own a 32x32 accumulator (16 f32 AGPR/VGPR per lane).
// Within a K-step the 32 k's are split 16/16 over the two lane halves that
// the MFMA's A/B operand maps assign to k = 0 / 1, so each lane reads its 16
// operand floats with four ds_read_b128 from a row-major [row][32+4] LDS tile
// (the +4 pad makes any 16 consecutive rows hit distinct 16-B bank slots).
// Global -> LDS staging is register double-buffered: the next K-step's loads
// are issued before the current step's MFMAs and written to the other LDS
// buffer afterwards; one barrier per K-step.
#include "common.hpp"

namespace raft {
namespace {

constexpr int BM = 64;
constexpr int BN = 64;
constexpr int BK = 32;
constexpr int LDSK = BK + 4;

struct ConvArgs {
  raft_conv2d_params p;
  int M;        // batch * out_h * out_w
  int K;        // packed row length (k_pad)
  int ctot;     // in0_c + in1_c
  int cpt;      // VEC: K-steps per tap (c_pad / BK)
  int taps;     // kh * kw
};

__device__ __forceinline__ float sigmoidf_(float v) { return 1.0f / (1.0f + expf(-v)); }

template <int MODE>
__device__ __forceinline__ void load_a(const ConvArgs& a, int kc, const int (&pb)[2], const int (&py)[2],
                                       const int (&px)[2], const bool (&pv)[2], int lq, f32x4 (&ra)[2]) {
  const raft_conv2d_params& p = a.p;
  if constexpr (MODE == RAFT_CONV_VEC) {
    const int tap = kc / a.cpt;
    const int c = (kc - tap * a.cpt) * BK + lq * 4;
    const int ky = tap / p.kw, kx = tap - ky * p.kw;
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      f32x4 v = {0.f, 0.f, 0.f, 0.f};
      const int iy = py[i] + ky, ix = px[i] + kx;
      if (pv[i] && iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w) {
        const long pix = ((long)pb[i] * p.in_h + iy) * p.in_w + ix;
        if (c < p.in0_c) {
          v = *reinterpret_cast<const f32x4*>(p.in0 + pix * p.in0_ld + c);
        } else if (c - p.in0_c < p.in1_c) {
          v = *reinterpret_cast<const f32x4*>(p.in1 + pix * p.in1_ld + (c - p.in0_c));
        }
      }
      ra[i] = v;
    }
  } else {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      float e[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int k = kc * BK + lq * 4 + j;
        const int tap = k / a.ctot;
        const int c = k - tap * a.ctot;
        float v = 0.f;
        if (pv[i] && tap < a.taps) {
          const int ky = tap / p.kw, kx = tap - ky * p.kw;
          const int iy = py[i] + ky, ix = px[i] + kx;
          if (iy >= 0 && iy < p.in_h && ix >= 0 && ix < p.in_w) {
            const long pix = ((long)pb[i] * p.in_h + iy) * p.in_w + ix;
            v = (c < p.in0_c) ? p.in0[pix * p.in0_ld + c] : p.in1[pix * p.in1_ld + (c - p.in0_c)];
          }
        }
        e[j] = v;
      }
      ra[i] = f32x4{e[0], e[1], e[2], e[3]};
    }
  }
}

template <int MODE>
__global__ __launch_bounds__(256) void conv_gemm_kernel(ConvArgs a) {
  __shared__ __attribute__((aligned(16))) float smem[2 * (BM + BN) * LDSK];
  // buffer b: A tile at smem + b*STAGE, B tile right after it
  constexpr int STAGE = (BM + BN) * LDSK;
  const raft_conv2d_params& p = a.p;

  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int m0 = blockIdx.x * BM;
  const int n0 = blockIdx.y * BN;

  // staging assignment: rows lr and lr+32, 4-float quad lq of the 32-float K-step
  const int lr = tid >> 3, lq = tid & 7;
  int pb[2], py[2], px[2];
  bool pv[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + lr + 32 * i;
    pv[i] = m < a.M;
    const int mm = pv[i] ? m : 0;
    const int ox = mm % p.out_w;
    const int t = mm / p.out_w;
    const int oy = t % p.out_h;
    pb[i] = t / p.out_h;
    py[i] = oy * p.stride_h - p.pad_h;
    px[i] = ox * p.stride_w - p.pad_w;
  }
  const float* wrow0 = p.weight + (long)(n0 + lr) * a.K + lq * 4;
  const float* wrow1 = wrow0 + 32L * a.K;

  f32x4 ra[2], rb[2];
  const int nk = a.K / BK;

  auto stage_store = [&](int buf) {
    float* A = smem + buf * STAGE;
    float* B = A + BM * LDSK;
    *reinterpret_cast<f32x4*>(A + lr * LDSK + lq * 4) = ra[0];
    *reinterpret_cast<f32x4*>(A + (lr + 32) * LDSK + lq * 4) = ra[1];
    *reinterpret_cast<f32x4*>(B + lr * LDSK + lq * 4) = rb[0];
    *reinterpret_cast<f32x4*>(B + (lr + 32) * LDSK + lq * 4) = rb[1];
  };

  load_a<MODE>(a, 0, pb, py, px, pv, lq, ra);
  rb[0] = *reinterpret_cast<const f32x4*>(wrow0);
  rb[1] = *reinterpret_cast<const f32x4*>(wrow1);
  stage_store(0);
  __syncthreads();

  f32x16 acc = {};
  const int arow = (wm * 32 + (lane & 31)) * LDSK + (lane >> 5) * 16;
  const int brow = (wn * 32 + (lane & 31)) * LDSK + (lane >> 5) * 16;

  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    const bool more = kc + 1 < nk;
    if (more) {
      load_a<MODE>(a, kc + 1, pb, py, px, pv, lq, ra);
      rb[0] = *reinterpret_cast<const f32x4*>(wrow0 + (kc + 1) * BK);
      rb[1] = *reinterpret_cast<const f32x4*>(wrow1 + (kc + 1) * BK);
    }
    const float* A = smem + cur * STAGE;
    const float* B = A + BM * LDSK;
    f32x4 av[4], bv[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      av[j] = *reinterpret_cast<const f32x4*>(A + arow + 4 * j);
      bv[j] = *reinterpret_cast<const f32x4*>(B + brow + 4 * j);
    }
#pragma unroll
    for (int s = 0; s < 16; ++s) {
      acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s >> 2][s & 3], bv[s >> 2][s & 3], acc, 0, 0, 0);
    }
    if (more) stage_store(cur ^ 1);
    __syncthreads();
  }

  // ---- epilogue: lane owns column n, rows (r&3) + 8*(r>>2) + 4*(lane>>5)
  const int n = n0 + wn * 32 + (lane & 31);
  if (n >= p.n) return;
  const float bias = p.bias ? p.bias[n] : 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = m0 + wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    if (m >= a.M) continue;
    const float v = acc[r] + bias;
    float* o = p.out + (long)m * p.out_ld + n;
    switch (p.epilogue) {
      case RAFT_EPI_LINEAR:
        *o = p.alpha * v;
        break;
      case RAFT_EPI_RELU:
        *o = fmaxf(v, 0.f);
        break;
      case RAFT_EPI_RESID_RELU:
        *o = fmaxf(p.aux0[(long)m * p.aux0_ld + n] + fmaxf(v, 0.f), 0.f);
        break;
      case RAFT_EPI_GRU_ZR:
        if (n < p.split) {
          *o = sigmoidf_(v);
        } else {
          const int c = n - p.split;
          p.out1[(long)m * p.out1_ld + c] = sigmoidf_(v) * p.aux0[(long)m * p.aux0_ld + c];
        }
        break;
      case RAFT_EPI_GRU_Q: {
        const float q = tanhf(v);
        const float z = p.aux1[(long)m * p.aux1_ld + n];
        const float h = p.aux0[(long)m * p.aux0_ld + n];
        *o = (1.0f - z) * h + z * q;
        break;
      }
      case RAFT_EPI_TANH_RELU:
        if (n < p.split)
          *o = tanhf(v);
        else
          p.out1[(long)m * p.out1_ld + (n - p.split)] = fmaxf(v, 0.f);
        break;
      case RAFT_EPI_ADD_TO_OUT:
        *o = *o + v;
        break;
      default:
        break;
    }
  }
}

}  // namespace
}  // namespace raft

using namespace raft;

extern "C" int raft_conv2d_packed_shape(int mode, int n, int kh, int kw, int cin, int* n_pad, int* k_pad) {
  RAFT_REQUIRE(n > 0 && kh > 0 && kw > 0 && cin > 0 && n_pad && k_pad, "raft_conv2d_packed_shape: bad args");
  *n_pad = round_up(n, BN);
  if (mode == RAFT_CONV_VEC)
    *k_pad = kh * kw * round_up(cin, BK);
  else if (mode == RAFT_CONV_GATHER)
    *k_pad = round_up(kh * kw * cin, BK);
  else
    return set_error(RAFT_E_INVALID, "raft_conv2d_packed_shape: unknown mode %d", mode);
  return 0;
}

extern "C" int raft_conv2d(const raft_conv2d_params* pp, raft_stream_t stream) {
  RAFT_REQUIRE(pp != nullptr, "raft_conv2d: null params");
  const raft_conv2d_params& p = *pp;
  RAFT_REQUIRE(p.in0 && p.weight && p.out, "raft_conv2d: null in0/weight/out");
  RAFT_REQUIRE(p.batch > 0 && p.in_h > 0 && p.in_w > 0 && p.out_h > 0 && p.out_w > 0 && p.n > 0,
               "raft_conv2d: bad sizes");
  RAFT_REQUIRE(p.kh > 0 && p.kw > 0 && p.stride_h > 0 && p.stride_w > 0 && p.pad_h >= 0 && p.pad_w >= 0,
               "raft_conv2d: bad kernel geometry");
  RAFT_REQUIRE(p.out_h == (p.in_h + 2 * p.pad_h - p.kh) / p.stride_h + 1 &&
                   p.out_w == (p.in_w + 2 * p.pad_w - p.kw) / p.stride_w + 1,
               "raft_conv2d: out_h/out_w inconsistent with input and kernel geometry");
  RAFT_REQUIRE(p.in0_c > 0 && p.in1_c >= 0 && (p.in1_c == 0 || p.in1), "raft_conv2d: bad segments");
  RAFT_REQUIRE(p.in0_ld >= p.in0_c && (p.in1_c == 0 || p.in1_ld >= p.in1_c) && p.out_ld >= 1,
               "raft_conv2d: leading dimension smaller than channel count");
  const int ctot = p.in0_c + p.in1_c;
  ConvArgs a;
  a.p = p;
  a.M = p.batch * p.out_h * p.out_w;
  a.ctot = ctot;
  a.taps = p.kh * p.kw;
  int n_pad = 0, k_pad = 0;
  int rc = raft_conv2d_packed_shape(p.mode, p.n, p.kh, p.kw, ctot, &n_pad, &k_pad);
  if (rc) return rc;
  a.K = k_pad;
  a.cpt = round_up(ctot, BK) / BK;
  if (p.mode == RAFT_CONV_VEC) {
    RAFT_REQUIRE(p.in0_c % 4 == 0 && p.in1_c % 4 == 0, "raft_conv2d VEC: channel counts must be multiples of 4");
    RAFT_REQUIRE(p.in1_c == 0 || p.in0_c % BK == 0, "raft_conv2d VEC: seg0 channels must be a multiple of 32 with seg1");
    RAFT_REQUIRE(p.in0_ld % 4 == 0 && (p.in1_c == 0 || p.in1_ld % 4 == 0), "raft_conv2d VEC: ld must be a multiple of 4");
    RAFT_REQUIRE(((uintptr_t)p.in0 & 15) == 0 && ((uintptr_t)p.in1 & 15) == 0,
                 "raft_conv2d VEC: inputs must be 16-byte aligned");
  }
  RAFT_REQUIRE(((uintptr_t)p.weight & 15) == 0, "raft_conv2d: weight must be 16-byte aligned");
  switch (p.epilogue) {
    case RAFT_EPI_RESID_RELU:
      RAFT_REQUIRE(p.aux0, "raft_conv2d: RESID_RELU needs aux0");
      break;
    case RAFT_EPI_GRU_ZR:
      RAFT_REQUIRE(p.aux0 && p.out1 && p.split > 0 && p.split < p.n, "raft_conv2d: GRU_ZR needs aux0, out1, split");
      break;
    case RAFT_EPI_GRU_Q:
      RAFT_REQUIRE(p.aux0 && p.aux1, "raft_conv2d: GRU_Q needs aux0 (h) and aux1 (z)");
      break;
    case RAFT_EPI_TANH_RELU:
      RAFT_REQUIRE(p.out1 && p.split > 0 && p.split < p.n, "raft_conv2d: TANH_RELU needs out1 and split");
      break;
    case RAFT_EPI_LINEAR:
    case RAFT_EPI_RELU:
    case RAFT_EPI_ADD_TO_OUT:
      break;
    default:
      return set_error(RAFT_E_INVALID, "raft_conv2d: unknown epilogue %d", p.epilogue);
  }
  dim3 grid(cdiv(a.M, BM), n_pad / BN);
  hipStream_t s = as_stream(stream);
  if (p.mode == RAFT_CONV_VEC)
    hipLaunchKernelGGL(conv_gemm_kernel<RAFT_CONV_VEC>, grid, dim3(256), 0, s, a);
  else
    hipLaunchKernelGGL(conv_gemm_kernel<RAFT_CONV_GATHER>, grid, dim3(256), 0, s, a);
  return check_launch("raft_conv2d");
}
