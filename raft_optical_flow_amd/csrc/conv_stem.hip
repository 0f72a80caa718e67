// The encoders' stem: a 7x7 / stride-2 / pad-3 convolution of the 3-channel prepared images
// (BasicEncoder.conv1, core/extractor.py:128, 136; SmallEncoder.conv1 :200), gfx950.
//
// The generic GEMM's GATHER mode fetched every (tap, channel) element of a 147-wide K through a
// per-element index table: 4-B loads, ~40 % of the encoder's first milliseconds in one conv.  Here
// a work-group owns 8x16 output pixels x all 64 outputs and stages its input patch ONCE:
// (2*8+5) x (2*16+5) pixels x 3 channels = 9.3 KB of fp32 in LDS, read as contiguous 111-float
// rows.  The im2col operand is never built: each MFMA lane reads its 8 K values of a fragment
// straight from the patch through a 160-entry offset table (k -> ky*111 + kx*3 + c, the GATHER
// packing's k order; the 13 K-padding entries clamp to a zero sentinel past the patch, never
// to LDS outside it), splits them to f16 hi | lo (or rounds to f16 / bf16) in registers, and
// multiplies them with the pre-split weight staged in LDS once per work-group (40 KB, XOR-
// swizzled rows).  Work-groups walk tiles (three per CU), so the weight staging is paid once
// per ~2 tiles at config 2; the epilogue: bias, linear or relu, the range guard.
#include "conv_common.hpp"

namespace raft {
namespace {

constexpr int ST_TH = 8, ST_TW = 16;                        // output tile
constexpr int ST_K = 7, ST_S = 2, ST_C = 3;                // 7x7, stride 2, 3 channels
constexpr int ST_PH = (ST_TH - 1) * ST_S + ST_K;           // 21 patch rows
constexpr int ST_PW = (ST_TW - 1) * ST_S + ST_K;           // 37 patch columns
constexpr int ST_ROW = ST_PW * ST_C;                       // 111 floats per patch row
constexpr int ST_PATCH = ST_PH * ST_ROW;                   // 2331 floats (+1 zero sentinel)
constexpr int ST_KS = 5;                                   // K = 147 -> 160 = 5 K-steps of 32
constexpr int ST_N = 64;                                   // outputs
constexpr int ST_WBYTES = ST_KS * ST_N * 128;              // split weight in LDS: 40 KB

struct StemArgs {
  raft_conv2d_params p;
  int tx_n, ty_n, ntiles;
  unsigned w_bytes;
};

template <int PREC>
__global__ __launch_bounds__(256, 3) void conv_stem_kernel(StemArgs sa) {  // 3 work-groups per CU
  constexpr bool X3 = PREC == RAFT_PREC_F16X3;
  constexpr bool BF = PREC == RAFT_PREC_BF16;
  const raft_conv2d_params& p = sa.p;
  __shared__ __attribute__((aligned(16))) char wlds[ST_WBYTES];
  __shared__ __attribute__((aligned(16))) float patch[ST_PATCH + 4];
  __shared__ __attribute__((aligned(16))) int koff[ST_KS * 32];
  const int tid = threadIdx.x, lane = tid & 63;
  const int w = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int m = lane & 31, h = lane >> 5;

  // the split weight [n][160] (row n: 5 K-steps x 128 B) -> LDS [j][n][128 B], quads XOR-swizzled by n
  for (int i = tid; i < ST_WBYTES / 16; i += 256) {
    const int n = i / (ST_KS * 8), rest = i - n * (ST_KS * 8), j = rest >> 3, q = rest & 7;
    const f32x4 v = *reinterpret_cast<const f32x4*>(reinterpret_cast<const char*>(p.weight) + (long)i * 16);
    *reinterpret_cast<f32x4*>(wlds + (j * ST_N + n) * 128 + ((q ^ ((n >> 1) & 7)) << 4)) = v;
  }
  // k = (ky*7 + kx)*3 + c -> its patch offset; K padding -> the zero sentinel past the patch
  for (int k = tid; k < ST_KS * 32; k += 256) {
    const int t = k / ST_C, c = k - t * ST_C, ky = t / ST_K, kx = t - ky * ST_K;
    koff[k] = k < ST_K * ST_K * ST_C ? ky * ST_ROW + kx * ST_C + c : ST_PATCH;
  }
  if (tid == 0) patch[ST_PATCH] = 0.f;

  const int in_h = p.in_h, in_w = p.in_w;
  const float* in = p.in0;
  const int ld = p.in0_ld;
  const int per = sa.tx_n * sa.ty_n;
  const int bsw = (m >> 1) & 7;
  for (int tile = blockIdx.x; tile < sa.ntiles; tile += gridDim.x) {
    const int b = tile / per, sr = tile - b * per;
    const int oy0 = (sr / sa.tx_n) * ST_TH, ox0 = (sr % sa.tx_n) * ST_TW;
    const int iy0 = oy0 * ST_S - p.pad_h, ix0 = ox0 * ST_S - p.pad_w;
    __syncthreads();  // the previous tile's patch reads are done (and, first time, the staging above)
    // the input patch: row r = 37 pixels x 3 channels (zeros off the image)
#ifndef STEM_PIX
#define STEM_PIX 1
#endif
    if (STEM_PIX && ld == ST_C) {
      // one pixel's 3 channels per thread and step (777 per tile: 3 pixels per thread instead of 9
      // scalar loads with their index arithmetic), zeros off the image by an out-of-range offset
      const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
          const_cast<float*>(in), (short)0, (int)((unsigned)(p.batch * in_h * in_w) * 12u), 0x00020000);
      for (int i = tid; i < ST_PH * ST_PW; i += 256) {
        const int r = i / ST_PW, px = i - r * ST_PW;
        const int yy = iy0 + r, xx = ix0 + px;
        const bool ok = (unsigned)yy < (unsigned)in_h && (unsigned)xx < (unsigned)in_w;
        const unsigned off = ok ? (unsigned)((b * in_h + yy) * in_w + xx) * 12u : 0x80000000u;
        // (8 + 4 B: the 12-B buffer-load builtin came out as one dword, replicated, with this compiler)
        const f32x2 v01 = __builtin_bit_cast(f32x2, __builtin_amdgcn_raw_buffer_load_b64(rs, off, 0, 0));
        const float v2 = __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(rs, off, 8, 0));
        float* d = patch + r * ST_ROW + px * ST_C;
        d[0] = v01[0];
        d[1] = v01[1];
        d[2] = v2;
      }
    } else
    for (int i = tid; i < ST_PATCH; i += 256) {
      const int r = i / ST_ROW, e = i - r * ST_ROW, px = e / ST_C, c = e - px * ST_C;
      const int yy = iy0 + r, xx = ix0 + px;
      float v = 0.f;
#ifndef STEM_ABL_NOPATCH  // (dev ablation: no input loads, wrong results)
      if ((unsigned)yy < (unsigned)in_h && (unsigned)xx < (unsigned)in_w)
        v = in[((long)b * in_h * in_w + (long)yy * in_w + xx) * ld + c];
#endif
      patch[i] = v;
    }
    __syncthreads();
    // wave w: output rows 2w, 2w+1 (32 pixels) x 64 outputs; lane m = pixel (row 2w + m/16, col m%16)
    const int py = 2 * w + (m >> 4), px = m & 15;
    // the lane's window origin in the patch; a K-padding entry (koff = ST_PATCH) clamps to the
    // zero sentinel (every real tap lies below it: base + koff <= ST_PATCH - 1)
    const int pbase = py * ST_S * ST_ROW + px * ST_S * ST_C;
    auto at = [&](int o) { return patch[min(pbase + o, ST_PATCH)]; };
    f32x16 acc[2] = {}, accx[2] = {};
#pragma unroll
    for (int j = 0; j < ST_KS; ++j) {
      h8 ah[2], al[2];
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const int4 o0 = *reinterpret_cast<const int4*>(&koff[32 * j + 8 * (2 * h + qq)]);
        const int4 o1 = *reinterpret_cast<const int4*>(&koff[32 * j + 8 * (2 * h + qq) + 4]);
        const f32x4 x0 = {at(o0.x), at(o0.y), at(o0.z), at(o0.w)};
        const f32x4 x1 = {at(o1.x), at(o1.y), at(o1.z), at(o1.w)};
        split8<X3, BF>(x0, x1, ah[qq], al[qq]);
      }
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const char* brow = wlds + (j * ST_N + sb * 32 + m) * 128;
#pragma unroll
        for (int qq = 0; qq < 2; ++qq) {
          const h8 bh = *reinterpret_cast<const h8*>(brow + (((2 * h + qq) ^ bsw) << 4));
          if constexpr (BF) {
            acc[sb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, ah[qq]), __builtin_bit_cast(bf8, bh),
                                                              acc[sb], 0, 0, 0);
          } else {
            acc[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], bh, acc[sb], 0, 0, 0);
          }
          if constexpr (X3) {
            const h8 bl = *reinterpret_cast<const h8*>(brow + (((4 + 2 * h + qq) ^ bsw) << 4));
            accx[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], bl, accx[sb], 0, 0, 0);
            acc[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[qq], bh, acc[sb], 0, 0, 0);
          }
        }
      }
    }
    int rows[16];
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int oy = oy0 + 2 * w + (mm >> 4), ox = ox0 + (mm & 15);
      rows[r] = (oy < p.out_h && ox < p.out_w) ? (b * p.out_h + oy) * p.out_w + ox : -1;
    }
    // epilogue (the stem's: linear or relu, bias, range guard; InstanceNorm partials)
    if constexpr (X3) {
#pragma unroll
      for (int sb = 0; sb < 2; ++sb)
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[sb][r] += accx[sb][r] * (1.0f / SPLIT_SCALE);
    }
    const bool relu = p.epilogue == RAFT_EPI_RELU;
#pragma unroll
    for (int sb = 0; sb < 2; ++sb) {
      const int n = sb * 32 + m;
      const float bias = p.bias ? p.bias[n] : 0.f;
      bool big = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        float v = acc[sb][r] + bias;
        v = relu ? fmaxf(v, 0.f) : v;
        big |= rows[r] >= 0 && fabsf(v) > RAFT_RANGE_LIMIT;
#ifndef STEM_ABL_NOSTORE  // (dev ablation: no output stores, wrong results)
        if (rows[r] >= 0) p.out[(long)rows[r] * p.out_ld + n] = v;
#endif
      }
      if (p.range_flag && big) *p.range_flag = 1;
      if (p.stats_part) tile_stats(p, rows, n, acc[sb], (long)tile * 4 + w);
    }
  }
}

}  // namespace

namespace {
bool stem_covers(const raft_conv2d_params& p, int k_pad) {
  static const bool enabled = [] {
    const char* e = getenv("RAFT_CONV_STEM");
    return !(e && e[0] == '0');
  }();
  if (!enabled) return false;
  if (p.mode != RAFT_CONV_GATHER || p.kh != ST_K || p.kw != ST_K || p.stride_h != ST_S || p.stride_w != ST_S ||
      p.in0_c != ST_C || p.in1_c != 0 || p.n != ST_N || k_pad != ST_KS * 32)
    return false;
  if (p.precision != RAFT_PREC_F16X3 && p.precision != RAFT_PREC_F16 && p.precision != RAFT_PREC_BF16) return false;
  if ((p.epilogue != RAFT_EPI_LINEAR || p.alpha != 1.0f) && p.epilogue != RAFT_EPI_RELU) return false;
  if (p.add0) return false;
  return p.out_h == (p.in_h + 2 * p.pad_h - ST_K) / ST_S + 1 && p.out_w == (p.in_w + 2 * p.pad_w - ST_K) / ST_S + 1;
}
}  // namespace

int conv_stem_stats_slots(const raft_conv2d_params& p, int k_pad) {
  if (!stem_covers(p, k_pad)) return 0;
  return cdiv(p.out_w, ST_TW) * cdiv(p.out_h, ST_TH) * 4;
}

// The stem kernel when the conv is one it covers (GATHER packing, 7x7 / stride 2 / pad 3, 3 input
// channels, 64 outputs, a split-weight precision, an epilogue without a second input segment);
// returns 1 without launching otherwise.  Arguments are validated by raft_conv2d.
int conv_stem_launch(const raft_conv2d_params& p, int k_pad, hipStream_t s) {
  if (!stem_covers(p, k_pad)) return 1;
  StemArgs sa;
  sa.p = p;
  sa.tx_n = cdiv(p.out_w, ST_TW);
  sa.ty_n = cdiv(p.out_h, ST_TH);
  const long nt = (long)p.batch * sa.tx_n * sa.ty_n;
  if (nt >= (1L << 31)) return 1;
  sa.ntiles = (int)nt;
  // three work-groups per CU (LDS: 40 KB weight + 9.3 KB patch), each walking tiles
  const int grid = (int)(nt < 3 * 256 ? nt : 3 * 256);
  if (p.precision == RAFT_PREC_F16X3)
    hipLaunchKernelGGL(conv_stem_kernel<RAFT_PREC_F16X3>, dim3(grid), dim3(256), 0, s, sa);
  else if (p.precision == RAFT_PREC_F16)
    hipLaunchKernelGGL(conv_stem_kernel<RAFT_PREC_F16>, dim3(grid), dim3(256), 0, s, sa);
  else
    hipLaunchKernelGGL(conv_stem_kernel<RAFT_PREC_BF16>, dim3(grid), dim3(256), 0, s, sa);
  return 0;
}

}  // namespace raft
