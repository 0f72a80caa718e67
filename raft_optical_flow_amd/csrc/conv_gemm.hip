// Implicit-GEMM convolution on MFMA for gfx950.
//
// Replaces every nn.Conv2d of the RAFT update block (core/update.py:6-325) and
// encoders (core/extractor.py:6-267), with the surrounding elementwise work of
// the reference fused into the epilogue (ReLU, residual add, GRU gates and
// blend, tanh/relu split of the context net, coords1 += delta_flow).
//
// Layout: NHWC rows.  GEMM view: M = output pixels, N = output channels,
// K = (tap, channel).  Work-group tile 64(M) x 64(N), K-step 32; four waves in
// a 2x2 arrangement each own a 32x32 accumulator.  LDS rows are 32+4 dwords
// (the pad keeps 32 consecutive rows' 16-B reads on distinct bank slots).
//
// Arithmetic (template PREC, include/raft_hip.h):
//  * FP32: v_mfma_f32_32x32x2_f32; the 32 k of a K-step are split 16/16 over
//    the two lane halves that the operand maps assign to k = 0 / 1, so each
//    lane reads its 16 operand floats with four ds_read_b128.
//  * F16X3: the staging threads split every fp32 activation into f16 hi and
//    2048-scaled f16 lo (the weight arrives pre-split); an LDS row holds the
//    K-step's 32 hi then 32 lo halves (same 128 B).  Per K-step a wave issues
//    2 hi*hi MFMAs into acc and 4 cross MFMAs (hi*lo, lo*hi) into accx on
//    v_mfma_f32_32x32x16_f16 (16x the f32 rate): 6 x 32 cycles instead of
//    16 x 64.  Result acc + accx/2048: ~22-bit operands, fp32 accumulation.
//  * F16: hi*hi only (the mixed-precision mode).
//  * BF16: one bf16 product on v_mfma_f32_32x32x16_bf16 (bf16 mixed precision:
//    activations rounded to bf16 at staging, weights pre-converted).
//
// Pipeline: two register staging sets and two LDS buffers.  The global loads
// of K-step k+2 are issued right after the barrier that publishes step k+1,
// one barrier per K-step.  VEC staging uses raw buffer loads: per-tap row byte
// offsets (recomputed only when the K walk changes tap), the K-step's channel
// offset as the wave-uniform soffset, and out-of-image rows pointed past the
// buffer end so the hardware returns zeros (no branches, no 64-bit address
// arithmetic in the loop).  GATHER mode (inputs with < 4 or unaligned
// channels: the 3-channel stem, the 2-channel flow) decodes k -> (ky, kx, c)
// through a per-workgroup LDS table.
//
// N <= 4 outputs (the flow head's 256 -> 2 conv) use conv_smalln_kernel: one
// wave per output pixel, channels across lanes, wave reduction per output.
#include "conv_common.hpp"

namespace raft {
namespace {

constexpr int BM = 64;
constexpr int BN = 64;
constexpr int BK = 32;
constexpr int LDSK = BK + 4;
constexpr int STAGE = (BM + BN) * LDSK;       // floats per LDS buffer
constexpr int MAX_GATHER_K = 1024;
#ifndef CONV_SCHED
#define CONV_SCHED 1                              // sched_group_barrier interleave of a phase
#endif
#ifndef GEMM_NS
#define GEMM_NS 2                                 // staging register sets (NS-1 K-steps in flight + one refilling)
#endif            // k_pad limit of GATHER mode (LDS table)

struct ConvArgs {
  raft_conv2d_params p;
  int M;        // batch * out_h * out_w
  int K;        // packed row length (k_pad)
  int ctot;     // in0_c + in1_c
  int cpad;     // VEC: channels per tap in the packed weight (multiple of BK)
  int taps;     // kh * kw
  int gn;       // N-tiles
  unsigned w_bytes, in0_bytes, in1_bytes;  // buffer-descriptor ranges
  // InstanceNorm partials (p.stats_part, round 5): M tiled per image (tpi tiles of BM rows of one
  // image's hw output pixels, the last one ragged) so that each wave's 32 rows lie in one image; each
  // wave writes its (count, mean, M2) per column to slot 2 (image tile) + wm.  tpi = 0: M tiled flat
  int tpi, hw;
};

// Per-thread staging state: two A rows (output pixels) of the tile.
struct AWalk {
  int pb[2], py[2], px[2];  // pb: the row's image base pixel (b * in_h * in_w)
  bool pv[2];
};

// GATHER mode (small / unaligned inputs): element-wise loads through the
// k -> (ky, kx, c) LDS table, issued unconditionally from clamped addresses;
// returns the validity bits (bit 4*i + j), applied when staging.
__device__ __forceinline__ unsigned gather_a(const ConvArgs& a, const AWalk& w, int kc, int lq, const int* ktab,
                                             f32x4 (&ra)[2]) {
  const raft_conv2d_params& p = a.p;
  unsigned mask = 0;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    float e[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int code = ktab[kc * BK + lq * 4 + j];  // (ky << 20) | (kx << 10) | c, or -1 for padding
      const int ky = code >> 20, kx = (code >> 10) & 1023, c = code & 1023;
      const int iy = w.py[i] + ky, ix = w.px[i] + kx;
      const bool ok = w.pv[i] && code >= 0 && (unsigned)iy < (unsigned)p.in_h && (unsigned)ix < (unsigned)p.in_w;
      const long pix = (long)w.pb[i] + (long)iy * p.in_w + ix;
      const float* src = (c < p.in0_c) ? p.in0 + pix * p.in0_ld + c : p.in1 + pix * p.in1_ld + (c - p.in0_c);
      e[j] = *(ok ? src : p.in0);
      mask |= ok ? 1u << (4 * i + j) : 0u;
    }
    ra[i] = f32x4{e[0], e[1], e[2], e[3]};
  }
  return mask;
}

// KG = number of K-groups: the work-group holds KG x 4 waves; group g runs the
// K-steps g, g+KG, g+2KG, ... of the same 64x64 output tile with its own LDS
// double buffer, so each SIMD carries KG waves of the tile that interleave
// (one group's MFMAs cover the other's LDS reads, barrier skew and staging).
// The groups' accumulators are summed through LDS before the epilogue.
#ifdef STAMPS  // dev-only phase timing (tools/conv_bench.py STAMPS=1 with a -DSTAMPS variant)
__device__ unsigned long long g_stamp[4 * 16384];
__device__ __forceinline__ unsigned long long stamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif

template <int MODE, int KG, int PREC, int NS>
__global__ __launch_bounds__(256 * KG, 4) void conv_gemm_kernel(ConvArgs a) {  // 4 waves per SIMD: <= 128 VGPRs
  static_assert(NS >= 2, "at least two staging register sets");
  constexpr int U = NS % 2 ? 2 * NS : NS;  // phase unroll: static LDS-buffer parity and register-set index
  constexpr int D = NS - 1;                // K-steps in flight ahead of the one being staged
  __shared__ __attribute__((aligned(16))) float
      smem[KG * 2 * STAGE + (MODE == RAFT_CONV_GATHER ? MAX_GATHER_K : 0)];
  const raft_conv2d_params& p = a.p;
  const int tid = threadIdx.x;
  const int lane = tid & 63;
  const int wave = tid >> 6;
  const int g = __builtin_amdgcn_readfirstlane(wave >> 2);  // K-group (provably wave-uniform)
  const int wl = wave & 3;          // wave within the group
  const int wm = wl & 1, wn = wl >> 1;
  const int lt = tid & 255;         // thread within the group
  // 1-D grid of gm x gn tiles in XCD order, N fastest (an M-tile's N-tiles share its A rows)
  const int q = xcd_tile(blockIdx.x, gridDim.x);
  const int gn = a.gn;
  const int mt = q / gn;
  const int n0 = (q - mt * gn) * BN;
  int m0 = mt * BM, mlim = a.M;  // the tile's first row; rows from mlim on are outside it
  if (a.tpi > 0) {
    const int b = mt / a.tpi;
    m0 = b * a.hw + (mt - b * a.tpi) * BM;
    mlim = min(a.M, (b + 1) * a.hw);
  }
  int* ktab = reinterpret_cast<int*>(smem + KG * 2 * STAGE);
  float* gsm = smem + g * 2 * STAGE;  // this group's two LDS buffers

  if constexpr (MODE == RAFT_CONV_GATHER) {
    for (int k = tid; k < a.K; k += 256 * KG) {
      const int tap = k / a.ctot;
      const int c = k - tap * a.ctot;
      const int ky = tap / p.kw, kx = tap - ky * p.kw;
      ktab[k] = tap < a.taps ? ((ky << 20) | (kx << 10) | c) : -1;
    }
    __syncthreads();
  }

  // staging assignment: rows lr and lr+32, 4-float quad lq of the 32-float K-step
  const int lr = lt >> 3, lq = lt & 7;
  AWalk w;
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int m = m0 + lr + 32 * i;
    w.pv[i] = m < mlim;
    const int mm = w.pv[i] ? m : 0;
    const int ox = mm % p.out_w;
    const int t = mm / p.out_w;
    const int oy = t % p.out_h;
    w.pb[i] = (t / p.out_h) * p.in_h * p.in_w;
    w.py[i] = oy * p.stride_h - p.pad_h;
    w.px[i] = ox * p.stride_w - p.pad_w;
  }
  const int nk = a.K / BK;
  // wave-uniform operands, read once from the kernel arguments (readfirstlane'd
  // so the per-step selects stay scalar: no kernarg reloads, no waterfalls)
  const unsigned rfl_in0c = __builtin_amdgcn_readfirstlane(p.in0_c);
  const unsigned rfl_in1c = __builtin_amdgcn_readfirstlane(p.in1_c);
  const unsigned ld0b = __builtin_amdgcn_readfirstlane(p.in0_ld) * 4u;
  const unsigned ld1b = __builtin_amdgcn_readfirstlane(p.in1_c ? p.in1_ld : p.in0_ld) * 4u;
  const unsigned long long b0 = (unsigned long long)p.in0;
  const unsigned long long b1 = p.in1_c ? (unsigned long long)p.in1 : b0;
  const unsigned b0lo = __builtin_amdgcn_readfirstlane((unsigned)b0), b0hi = __builtin_amdgcn_readfirstlane((unsigned)(b0 >> 32));
  const unsigned b1lo = __builtin_amdgcn_readfirstlane((unsigned)b1), b1hi = __builtin_amdgcn_readfirstlane((unsigned)(b1 >> 32));
  const unsigned nrec0 = __builtin_amdgcn_readfirstlane(a.in0_bytes);
  const unsigned nrec1 = __builtin_amdgcn_readfirstlane(p.in1_c ? a.in1_bytes : a.in0_bytes);
  const int cpad = __builtin_amdgcn_readfirstlane(a.cpad);
  const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(p.weight, a.w_bytes);
  const unsigned wvoff0 = ((unsigned)(n0 + lr) * (unsigned)a.K + lq * 4) * 4u;
  const unsigned wvoff1 = wvoff0 + 32u * (unsigned)a.K * 4u;
  const int cnt = g < nk ? (nk - g + KG - 1) / KG : 0;  // this group's K-steps
  const int nj = (nk + KG - 1) / KG;                     // phases (group 0's count)
  f32x4 ra[NS][2], rb[NS][2];  // staging register sets: during phase t, steps t+1 .. t+D in flight, set t%NS refilling
  unsigned am[NS];             // their A validity masks

  // the K walk of issue(): this group's next K-step as (tap (ky, kx), first
  // channel cs) and weight byte offset, advanced incrementally in SGPRs
  // (issue() runs in step order); no branches, so a whole phase is one
  // scheduling region
  const int kw = __builtin_amdgcn_readfirstlane(p.kw);
  const unsigned in_h = __builtin_amdgcn_readfirstlane(p.in_h), in_w = __builtin_amdgcn_readfirstlane(p.in_w);
  int wcs = g * BK, wky = 0, wkx = 0;
  auto advance_tap = [&]() {
    const bool wrap = wcs >= cpad;
    wcs = wrap ? wcs - cpad : wcs;
    const int kx1 = wkx + (wrap ? 1 : 0);
    const bool row = kx1 == kw;
    wkx = row ? 0 : kx1;
    wky = row ? wky + 1 : wky;
  };
  advance_tap();
  advance_tap();
  unsigned wsoff = (unsigned)g * BK * 4u;
  int kstep = g;

  // issue() is unconditional: steps beyond this group's count load zeros
  // (offsets past the buffer ends), so every phase has the same load count
  // (hipcc's counted vmcnt stays exact) and the MFMA phases need no predicate
  auto issue = [&](f32x4(&ra)[2], f32x4(&rb)[2], unsigned& am) {
    if constexpr (MODE == RAFT_CONV_VEC) {
      const bool s0 = (unsigned)wcs < rfl_in0c;  // uniform: the K-step lies in segment 0
      const unsigned cl = (unsigned)(wcs + lq * 4);
      // channel limit of the K-step's segment (segment 1 starts at in0_c): one compare
      const unsigned lim = (kstep < nk) ? (s0 ? rfl_in0c : rfl_in0c + rfl_in1c) : 0u;
      const bool lane_ok = cl < lim;
      const unsigned soff = (unsigned)(s0 ? wcs : wcs - (int)rfl_in0c) * 4u;
      const unsigned blo = s0 ? b0lo : b1lo, bhi = s0 ? b0hi : b1hi, nrec = s0 ? nrec0 : nrec1;
      const unsigned ldb = s0 ? ld0b : ld1b;
      const __amdgpu_buffer_rsrc_t rs =
          make_rsrc(reinterpret_cast<const void*>(((unsigned long long)bhi << 32) | blo), nrec);
      // row byte offsets for this tap, 24-bit multiplies (pixels < 2^24, host-checked)
      unsigned voff[2];
#pragma unroll
      for (int i = 0; i < 2; ++i) {
        const int iy = w.py[i] + wky, ix = w.px[i] + wkx;
        const bool ok = lane_ok & w.pv[i] & ((unsigned)iy < in_h) & ((unsigned)ix < in_w);
        const unsigned pix = (unsigned)w.pb[i] + __umul24((unsigned)iy, in_w) + (unsigned)ix;
        voff[i] = ok ? __umul24(pix, ldb) + lq * 16u : OFF_INVALID;
      }
#ifdef ABL_NOLOAD  // timing ablation (dev builds only): no A/B global loads
      ra[0] = f32x4{(float)voff[0], 1.f, 2.f, 3.f};
      ra[1] = f32x4{(float)voff[1], 1.f, 2.f, (float)soff};
      (void)rs;
#else
      ra[0] = buf_load4(rs, voff[0], soff);
      ra[1] = buf_load4(rs, voff[1], soff);
#endif
      am = 0xFFu;
      wcs += KG * BK;
      advance_tap();
      advance_tap();
    } else {
      am = kstep < nk ? gather_a(a, w, kstep, lq, ktab, ra) : 0u;
    }
#ifdef ABL_NOLOAD
    rb[0] = f32x4{(float)wsoff, 1.f, 2.f, 3.f};
    rb[1] = f32x4{(float)wsoff, 1.f, 2.f, 4.f};
#else
    // past the last K-step the soffset points beyond the weight buffer: zeros
    const unsigned ws = kstep < nk ? wsoff : OFF_INVALID;
    rb[0] = buf_load4(rs_w, wvoff0, ws);
    rb[1] = buf_load4(rs_w, wvoff1, ws);
#endif
    wsoff += KG * BK * 4u;
    kstep += KG;
  };
  auto stage = [&](int buf, const f32x4(&ra)[2], const f32x4(&rb)[2], unsigned am) {
    float* A = gsm + buf * STAGE;
    float* B = A + BM * LDSK;
    f32x4 x0 = ra[0], x1 = ra[1];
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      x0[e] = (am >> e) & 1 ? x0[e] : 0.f;
      x1[e] = (am >> (4 + e)) & 1 ? x1[e] : 0.f;
    }
    if constexpr (PREC == RAFT_PREC_FP32) {
      *reinterpret_cast<f32x4*>(A + lr * LDSK + lq * 4) = x0;
      *reinterpret_cast<f32x4*>(A + (lr + 32) * LDSK + lq * 4) = x1;
    } else if constexpr (PREC == RAFT_PREC_BF16) {
      _Float16* a0 = reinterpret_cast<_Float16*>(A + lr * LDSK) + lq * 4;
      _Float16* a1 = reinterpret_cast<_Float16*>(A + (lr + 32) * LDSK) + lq * 4;
      *reinterpret_cast<h4*>(a0) = to_bf16x4(x0);
      *reinterpret_cast<h4*>(a1) = to_bf16x4(x1);
    } else {
      // row: 32 hi halves (bytes 0..63) then 32 lo halves (64..127)
      h4 h0, l0, h1, l1;
      split4(x0, h0, l0);
      split4(x1, h1, l1);
      _Float16* a0 = reinterpret_cast<_Float16*>(A + lr * LDSK) + lq * 4;
      _Float16* a1 = reinterpret_cast<_Float16*>(A + (lr + 32) * LDSK) + lq * 4;
      *reinterpret_cast<h4*>(a0) = h0;
      *reinterpret_cast<h4*>(a1) = h1;
      if constexpr (PREC == RAFT_PREC_F16X3) {
        *reinterpret_cast<h4*>(a0 + 32) = l0;
        *reinterpret_cast<h4*>(a1 + 32) = l1;
      }
    }
    // the weight block arrives in the LDS row format of its precision
    *reinterpret_cast<f32x4*>(B + lr * LDSK + lq * 4) = rb[0];
    *reinterpret_cast<f32x4*>(B + (lr + 32) * LDSK + lq * 4) = rb[1];
  };

  f32x16 acc = {};
  f32x16 accx = {};  // F16X3 cross terms (x 2048)
  const int arow = (wm * 32 + (lane & 31)) * LDSK + (lane >> 5) * 16;
  const int brow = (wn * 32 + (lane & 31)) * LDSK + (lane >> 5) * 16;
  auto compute = [&](int buf) {
    const float* A = gsm + buf * STAGE;
    const float* B = A + BM * LDSK;
    if constexpr (PREC == RAFT_PREC_FP32) {
      f32x4 av[4], bv[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        av[j] = *reinterpret_cast<const f32x4*>(A + arow + 4 * j);
        bv[j] = *reinterpret_cast<const f32x4*>(B + brow + 4 * j);
      }
#pragma unroll
      for (int s = 0; s < 16; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(av[s >> 2][s & 3], bv[s >> 2][s & 3], acc, 0, 0, 0);
    } else {
      // lane half h takes k in [16h, 16h+16): MFMA q gets k = 16h + 8q + j,
      // i.e. halves 8q.. of the lane's 16 (bytes 32h + 16q; lo at +64)
      const _Float16* Ar = reinterpret_cast<const _Float16*>(A + arow - (lane >> 5) * 8);
      const _Float16* Br = reinterpret_cast<const _Float16*>(B + brow - (lane >> 5) * 8);
      h8 ah[2], bh[2];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        ah[q] = *reinterpret_cast<const h8*>(Ar + 8 * q);
        bh[q] = *reinterpret_cast<const h8*>(Br + 8 * q);
      }
      if constexpr (PREC == RAFT_PREC_F16X3) {
        h8 al[2], bl[2];
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          al[q] = *reinterpret_cast<const h8*>(Ar + 32 + 8 * q);
          bl[q] = *reinterpret_cast<const h8*>(Br + 32 + 8 * q);
        }
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[q], bh[q], acc, 0, 0, 0);
          accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[q], bl[q], accx, 0, 0, 0);
          accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[q], bh[q], accx, 0, 0, 0);
        }
      } else if constexpr (PREC == RAFT_PREC_BF16) {
#pragma unroll
        for (int q = 0; q < 2; ++q)
          acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, ah[q]), __builtin_bit_cast(bf8, bh[q]),
                                                        acc, 0, 0, 0);
      } else {
#pragma unroll
        for (int q = 0; q < 2; ++q) acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[q], bh[q], acc, 0, 0, 0);
      }
    }
  };

  // one phase's schedule (LLVM sched groups): the LDS reads of the MFMA operands
  // first, then each MFMA followed by a share of the next stage's conversion
  // VALU and one of the global loads of step t+NS, then the LDS writes, so
  // the MFMA pipe is fed while the split runs and the loads queue at the
  // texture unit in the MFMA shadow (not all at once after the barrier)
  auto interleave = [&]() {
#if CONV_SCHED
    constexpr int NMF = PREC == RAFT_PREC_FP32 ? 16 : PREC == RAFT_PREC_F16X3 ? 6 : 2;
    constexpr int NRD = (PREC == RAFT_PREC_F16 || PREC == RAFT_PREC_BF16) ? 4 : 8;
    constexpr int NVA = PREC == RAFT_PREC_FP32 ? 1 : PREC == RAFT_PREC_F16X3 ? 6 : 10;
    // operand reads in two halves (the second half after a third of the
    // MFMAs) keep fewer fragment registers live
    __builtin_amdgcn_sched_group_barrier(0x100, NRD / 2, 0);
#pragma unroll
    for (int i = 0; i < NMF; ++i) {
      if (i == (NMF + 2) / 3) __builtin_amdgcn_sched_group_barrier(0x100, NRD - NRD / 2, 0);
      __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      __builtin_amdgcn_sched_group_barrier(0x2, NVA, 0);
      if (i < 4) __builtin_amdgcn_sched_group_barrier(0x20, 1, 0);  // the next step's global loads
    }
    __builtin_amdgcn_sched_group_barrier(0x200, 4, 0);
#endif
  };

#ifdef ABL_EMPTY
  if (a.M > 0) return;
#endif
#ifdef ABL_NOLOOP
  if (a.M > 0) {
    int rows[16];
    for (int r = 0; r < 16; ++r) rows[r] = -1;
    tile_epilogue(p, rows, n0 + wn * 32 + (lane & 31), acc);
    return;
  }
#endif
  // prologue: K-steps 0 .. NS-1 issued into sets 0 .. NS-1, step 0 staged
#pragma unroll
  for (int u = 0; u < NS; ++u) issue(ra[u], rb[u], am[u]);
  stage(0, ra[0], rb[0], am[0]);
  __syncthreads();

  // phase t: refill set t%NS (its step t was staged in phase t-1) with step
  // t+NS; MFMAs on LDS buffer t&1 (step t); stage step t+1 from set (t+1)%NS
  // into the other buffer; one barrier.  The refill has no dependence on the
  // rest of the phase, so the sched groups spread its loads between the
  // MFMAs.  The body is unrolled U times (static set index and buffer parity)
  // and is branch-free; hipcc's counted vmcnt keeps D steps in flight.  The
  // < U tail phases issue only the steps still needed.
  const int nfull = nj - nj % U;
#ifdef STAMPS
  unsigned long long st_work = 0, st_bar = 0, st_iss = 0, st0 = stamp_now();
  const unsigned long long st_begin = st0;
#endif
  for (int j = 0; j < nfull; j += U) {
#pragma unroll
    for (int u = 0; u < U; ++u) {
      issue(ra[u % NS], rb[u % NS], am[u % NS]);
#ifndef ABL_NOCOMPUTE
      compute(u & 1);
#endif
      stage((u + 1) & 1, ra[(u + 1) % NS], rb[(u + 1) % NS], am[(u + 1) % NS]);
      interleave();
#ifdef STAMPS
      const unsigned long long st1 = stamp_now();
      st_work += st1 - st0;
#endif
#ifndef ABL_NOBARRIER
      __syncthreads();
#endif
#ifdef STAMPS
      st0 = stamp_now();
      st_bar += st0 - st1;
#endif
    }
  }
#ifdef STAMPS
  {
    const unsigned wid = blockIdx.x * (KG * 4) + wave;
    if (lane == 0 && wid < 16384) {
      g_stamp[wid * 4 + 0] = st_work;
      g_stamp[wid * 4 + 1] = st_bar;
      g_stamp[wid * 4 + 2] = st_iss;
      g_stamp[wid * 4 + 3] = st0 - st_begin;
    }
  }
#endif
#pragma unroll
  for (int u = 0; u < U - 1; ++u) {
    const int t = nfull + u;
    if (t < nj) {
      if (t + NS < nj) issue(ra[u % NS], rb[u % NS], am[u % NS]);  // steps still to come
      compute(u & 1);
      if (t + 1 < nj) {
        stage((u + 1) & 1, ra[(u + 1) % NS], rb[(u + 1) % NS], am[(u + 1) % NS]);
        __syncthreads();
      }
    }
  }
  if constexpr (PREC == RAFT_PREC_F16X3) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += accx[r] * (1.0f / SPLIT_SCALE);
  }

  if constexpr (KG > 1) {
    // sum the K-groups' accumulators through LDS: red[r][wave-in-group][lane]
    __syncthreads();
    float* red = smem;
    for (int gg = 1; gg < KG; ++gg) {
      if (g == gg) {
#pragma unroll
        for (int r = 0; r < 16; ++r) red[(r * 4 + wl) * 64 + lane] = acc[r];
      }
      __syncthreads();
      if (g == 0) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[r] += red[(r * 4 + wl) * 64 + lane];
      }
      __syncthreads();
    }
    if (g != 0) return;
  }

  // ---- epilogue: lane owns column n, rows (r&3) + 8*(r>>2) + 4*(lane>>5)
  int rows[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int m = (int)row_of(m0 + wm * 32 + 4 * (lane >> 5), r);
    rows[r] = m < mlim ? m : -1;
  }
  if (p.stats_part) tile_stats(p, rows, n0 + wn * 32 + (lane & 31), acc, 2L * mt + wm);
  tile_epilogue(p, rows, n0 + wn * 32 + (lane & 31), acc);
}

// Small-N convolution (N <= 4, VEC inputs): one wave per output pixel.
template <int NOUT>
__global__ __launch_bounds__(256) void conv_smalln_kernel(ConvArgs a) {
  const raft_conv2d_params& p = a.p;
  const int lane = threadIdx.x & 63;
  const long m = (long)blockIdx.x * 4 + (threadIdx.x >> 6);
  if (m >= a.M) return;
  const int ox = m % p.out_w;
  const long t = m / p.out_w;
  const int oy = t % p.out_h;
  const int b = t / p.out_h;
  float acc[NOUT];
#pragma unroll
  for (int j = 0; j < NOUT; ++j) acc[j] = 0.f;
  for (int ky = 0; ky < p.kh; ++ky) {
    const int iy = oy * p.stride_h - p.pad_h + ky;
    if ((unsigned)iy >= (unsigned)p.in_h) continue;
    for (int kx = 0; kx < p.kw; ++kx) {
      const int ix = ox * p.stride_w - p.pad_w + kx;
      if ((unsigned)ix >= (unsigned)p.in_w) continue;
      const long pix = ((long)b * p.in_h + iy) * p.in_w + ix;
      const float* wt = p.weight + (ky * p.kw + kx) * a.cpad;
      for (int c = lane * 4; c < a.ctot; c += 256) {
        const f32x4 v = c < p.in0_c ? *reinterpret_cast<const f32x4*>(p.in0 + pix * p.in0_ld + c)
                                    : *reinterpret_cast<const f32x4*>(p.in1 + pix * p.in1_ld + (c - p.in0_c));
#pragma unroll
        for (int j = 0; j < NOUT; ++j) {
          const f32x4 wv = *reinterpret_cast<const f32x4*>(wt + (long)j * a.K + c);
          acc[j] += v[0] * wv[0] + v[1] * wv[1] + v[2] * wv[2] + v[3] * wv[3];
        }
      }
    }
  }
#pragma unroll
  for (int j = 0; j < NOUT; ++j) {
#pragma unroll
    for (int off = 32; off >= 1; off >>= 1) acc[j] += __shfl_xor(acc[j], off);
  }
  if (lane < p.n) {
    float v = acc[0];
#pragma unroll
    for (int j = 1; j < NOUT; ++j)
      if (lane == j) v = acc[j];
    epilogue(p, m, lane, v + (p.bias ? p.bias[lane] : 0.f));
  }
}

// Small-N 3x3 "same" convolution (the flow head's 256 -> 2 conv, core/update.py:6-16)
// over TH x 16 output tiles (4x16, or 2x16 when 4x16 tiles would leave CUs
// idle: config 2 at B = 1 has 112): one 512-thread work-group per tile; wave w owns the
// input channels 32w + 256k.  Lane (q, pb) = (lane & 7, lane >> 3) holds the
// weights of channel quad q for all 9 taps in registers (loaded with the
// patch: one memory round trip, no scalar-load chain) and accumulates the
// TH*2 pixels of block pb (4x16: tile row pb/2, columns 8(pb%2) .. +7) over its
// 4 channels; the (TH+2)x18 input patch is staged in LDS as [channel quad][patch
// pixel] (row stride padded to 109 pixels).  Partial sums meet through lane
// shuffles (the 8 quads) and LDS (the 8 waves) in a fixed order.
#ifndef SN_TH4_MIN_TILES  // dev builds: 0 = always 4x16 tiles
// 256 (one round; 512 until r04k: config 5's 510 4x16 tiles vs 1020 2x16 ones, 47.9 / 48.0 -> 48.3 / 48.4
// pairs/s on one box); RAFT_SN_TH4_MIN overrides
#define SN_TH4_MIN_TILES 256
#endif
// TH x 16 output tiles (TH = 4 or 2); SN_PXB = TH*16/8 pixels per lane block
template <int TH>
struct SnGeom {
  static constexpr int TW = 16, PH = TH + 2, PW = TW + 2, NP = PH * PW;
  static constexpr int QS = NP + 1;        // patch stride per channel quad (f32x4 elements)
  static constexpr int PXB = TH * TW / 8;  // pixels per lane block
  static constexpr int BPR = TW / PXB;     // lane blocks per tile row
};

template <int NOUT, int TH>
__global__ __launch_bounds__(512) void conv_smalln3x3_kernel(ConvArgs a, const float* __restrict__ wt) {
  using G = SnGeom<TH>;
  constexpr int SN_TH = TH, SN_TW = G::TW, SN_PW = G::PW, SN_NP = G::NP, SN_QS = G::QS, PXB = G::PXB;
  __shared__ f32x4 patch[8][8 * SN_QS];
  __shared__ float red[8][NOUT][64];
  const raft_conv2d_params& p = a.p;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tx_n = (p.out_w + SN_TW - 1) / SN_TW, ty_n = (p.out_h + SN_TH - 1) / SN_TH;
  const int per = tx_n * ty_n;
  const int b = blockIdx.x / per, sr = blockIdx.x - b * per;
  const int y0 = (sr / tx_n) * SN_TH, x0 = (sr % tx_n) * SN_TW;
  const long pbase = (long)b * p.in_h * p.in_w;
  const int q = lane & 7, pb = lane >> 3;
  const int prow = pb / G::BPR, pcol = PXB * (pb % G::BPR);  // the block's first output pixel in the tile
  float acc[PXB][NOUT];
#pragma unroll
  for (int i = 0; i < PXB; ++i)
#pragma unroll
    for (int j = 0; j < NOUT; ++j) acc[i][j] = 0.f;
  // ADD_TO_OUT (coords1 += delta_flow): the destination value loaded here, with the patch, not after
  // the reduction (one memory round trip fewer on the kernel's path)
#ifndef SN_PRE
#define SN_PRE 1
#endif
  const bool pre_on = SN_PRE && p.epilogue == RAFT_EPI_ADD_TO_OUT && !p.add0;
  const int ej = threadIdx.x >> 6;
  const int ey = y0 + (lane >> 4), ex = x0 + (lane & 15);
  const bool eok = threadIdx.x < 64 * NOUT && ej < p.n && lane < SN_TH * SN_TW && ey < p.out_h && ex < p.out_w;
  const long em = ((long)b * p.out_h + ey) * p.out_w + ex;
  float pre = 0.f;
  if (pre_on && eok) pre = p.out[em * p.out_ld + ej];
  for (int cg = 32 * w; cg < a.ctot; cg += 256) {
    // weights of this lane's quad (zero-padded to cpad in the packed matrix)
    f32x4 wr[9][NOUT];
#pragma unroll
    for (int t = 0; t < 9; ++t)
#pragma unroll
      for (int j = 0; j < NOUT; ++j)
        wr[t][j] = *reinterpret_cast<const f32x4*>(wt + (long)j * a.K + t * a.cpad + cg + 4 * q);
    // stage: piece i = (patch pixel i >> 3, channel quad i & 7); zeros outside the image
    f32x4 v[(SN_NP * 8 + 63) / 64];
#pragma unroll
    for (int k = 0; k < (SN_NP * 8 + 63) / 64; ++k) {
      const int i = lane + 64 * k;
      const int pp = i >> 3, qq = i & 7;
      const int py = pp / SN_PW, px = pp - py * SN_PW;
      const int iy = y0 + py - 1, ix = x0 + px - 1;
      const int c = cg + 4 * qq;
      const bool ok = i < SN_NP * 8 && (unsigned)iy < (unsigned)p.in_h && (unsigned)ix < (unsigned)p.in_w && c < a.ctot;
      const long pix = pbase + (long)(ok ? iy : 0) * p.in_w + (ok ? ix : 0);
      const float* src = c < p.in0_c ? p.in0 + pix * p.in0_ld + c : p.in1 + pix * p.in1_ld + (c - p.in0_c);
      v[k] = ok ? *reinterpret_cast<const f32x4*>(src) : f32x4{0.f, 0.f, 0.f, 0.f};
    }
#pragma unroll
    for (int k = 0; k < (SN_NP * 8 + 63) / 64; ++k) {
      const int i = lane + 64 * k;
      if (i < SN_NP * 8) patch[w][(i & 7) * SN_QS + (i >> 3)] = v[k];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    const f32x4* pq = &patch[w][q * SN_QS];
#pragma unroll
    for (int ky = 0; ky < 3; ++ky)
#pragma unroll
      for (int kx = 0; kx < 3; ++kx)
#pragma unroll
        for (int i = 0; i < PXB; ++i) {
          const f32x4 x = pq[(prow + ky) * SN_PW + pcol + i + kx];
#pragma unroll
          for (int j = 0; j < NOUT; ++j) {
            const f32x4 wv = wr[ky * 3 + kx][j];
            acc[i][j] = fmaf(x[0], wv[0], acc[i][j]);
            acc[i][j] = fmaf(x[1], wv[1], acc[i][j]);
            acc[i][j] = fmaf(x[2], wv[2], acc[i][j]);
            acc[i][j] = fmaf(x[3], wv[3], acc[i][j]);
          }
        }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  }
  // the 8 channel quads of a pixel block: lanes q = 0..7 (xor 1, 2, 4)
#pragma unroll
  for (int i = 0; i < PXB; ++i)
#pragma unroll
    for (int j = 0; j < NOUT; ++j) {
      float t = acc[i][j];
      t += __shfl_xor(t, 1);
      t += __shfl_xor(t, 2);
      t += __shfl_xor(t, 4);
      acc[i][j] = t;
    }
  if (q == 0) {
#pragma unroll
    for (int i = 0; i < PXB; ++i)
#pragma unroll
      for (int j = 0; j < NOUT; ++j) red[w][j][prow * SN_TW + pcol + i] = acc[i][j];
  }
  __syncthreads();
  if (threadIdx.x < 64 * NOUT) {
    const int j = ej;
    float v = 0.f;
#pragma unroll
    for (int k = 0; k < 8; ++k) v += red[k][j][lane];
    if (eok) {
      const float vb = v + (p.bias ? p.bias[j] : 0.f);
      if (pre_on)
        p.out[em * p.out_ld + j] = pre + vb;  // (epilogue's ADD_TO_OUT: *o + v)
      else
        epilogue(p, em, j, vb);
    }
  }
}

}  // namespace
}  // namespace raft

using namespace raft;

namespace {
template <int MODE, int PREC, int NSETS = MODE == RAFT_CONV_VEC ? GEMM_NS : 2>
void launch_gemm_p(const ConvArgs& a, dim3 grid, bool two, hipStream_t s) {
  if (two)
    hipLaunchKernelGGL((conv_gemm_kernel<MODE, 2, PREC, NSETS>), grid, dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((conv_gemm_kernel<MODE, 1, PREC, NSETS>), grid, dim3(256), 0, s, a);
}
template <int MODE>
void launch_gemm_m(const ConvArgs& a, dim3 grid, bool two, hipStream_t s) {
  switch (a.p.precision) {
    case RAFT_PREC_F16X3: launch_gemm_p<MODE, RAFT_PREC_F16X3>(a, grid, two, s); break;
    case RAFT_PREC_F16: launch_gemm_p<MODE, RAFT_PREC_F16>(a, grid, two, s); break;
    case RAFT_PREC_BF16: launch_gemm_p<MODE, RAFT_PREC_BF16>(a, grid, two, s); break;
    default: launch_gemm_p<MODE, RAFT_PREC_FP32>(a, grid, two, s); break;
  }
}
void launch_gemm(const ConvArgs& a, dim3 grid, bool two, hipStream_t s) {
  if (a.p.mode == RAFT_CONV_VEC)
    launch_gemm_m<RAFT_CONV_VEC>(a, grid, two, s);
  else
    launch_gemm_m<RAFT_CONV_GATHER>(a, grid, two, s);
}

// fp32 packed weight -> per (row, K-step): 32 f16 hi then 32 f16 lo (x 2048)
__global__ void split_weight_kernel(const float* __restrict__ w, _Float16* __restrict__ out, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float x = w[i];
  const _Float16 h = (_Float16)x;
  const long blk = i >> 5, k = i & 31;
  out[blk * 64 + k] = h;
  out[blk * 64 + 32 + k] = (_Float16)((x - (float)h) * SPLIT_SCALE);
}
// fp32 packed weight -> per (row, K-step): 32 bf16 hi then 32 bf16 lo = bf16(x - hi)
__global__ void split_weight_bf16_kernel(const float* __restrict__ w, __bf16* __restrict__ out, long total) {
  const long i = (long)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= total) return;
  const float x = w[i];
  const __bf16 h = (__bf16)x;
  const long blk = i >> 5, k = i & 31;
  out[blk * 64 + k] = h;
  out[blk * 64 + 32 + k] = (__bf16)(x - (float)h);
}
// fp32 packed weight -> the column-scaled split (raft_conv2d_split_weight_scaled): one block per row
__global__ __launch_bounds__(256) void split_weight_scaled_kernel(const float* __restrict__ w, _Float16* __restrict__ out,
                                                                  float* __restrict__ inv, int k_pad) {
  const int n = blockIdx.x;
  const float* row = w + (long)n * k_pad;
  float mx = 0.f;
  for (int k = threadIdx.x; k < k_pad; k += 256) mx = fmaxf(mx, fabsf(row[k]));
  __shared__ float red[4];
#pragma unroll
  for (int o = 32; o > 0; o >>= 1) mx = fmaxf(mx, __shfl_xor(mx, o));
  if ((threadIdx.x & 63) == 0) red[threadIdx.x >> 6] = mx;
  __syncthreads();
  mx = fmaxf(fmaxf(red[0], red[1]), fmaxf(red[2], red[3]));
  int e = 0;
  if (mx > 0.f) frexpf(mx, &e);  // mx = f * 2^e, f in [0.5, 1): mx < 2^e
  e = mx > 0.f ? max(min(14 - e, 100), -100) : 0;
  const float sc = ldexpf(1.0f, e);
  for (int k = threadIdx.x; k < k_pad; k += 256) {
    const float x = row[k] * sc;  // exact (a power of two, no overflow / underflow in range)
    const _Float16 h = (_Float16)x;
    const long blk = ((long)n * k_pad + k) >> 5, kk = k & 31;
    out[blk * 64 + kk] = h;
    out[blk * 64 + 32 + kk] = (_Float16)(x - (float)h);
  }
  if (threadIdx.x == 0) inv[n] = ldexpf(1.0f, -e);
}
}  // namespace

#ifdef STAMPS
extern "C" int raft_debug_stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_stamp), sizeof(unsigned long long) * (size_t)n);
}
#endif

extern "C" int raft_conv2d_split_weight(const float* w, void* out, int n_pad, int k_pad, raft_stream_t stream) {
  RAFT_REQUIRE(w && out && n_pad > 0 && k_pad > 0 && k_pad % BK == 0, "raft_conv2d_split_weight: bad args");
  RAFT_REQUIRE((const void*)w != out, "raft_conv2d_split_weight: in-place split is not supported");
  const long total = (long)n_pad * k_pad;
  hipLaunchKernelGGL(split_weight_kernel, dim3((unsigned)cdiv_l(total, 256)), dim3(256), 0, as_stream(stream), w,
                     reinterpret_cast<_Float16*>(out), total);
  return check_launch("raft_conv2d_split_weight");
}

extern "C" size_t raft_conv2d_split_scaled_bytes(int n_pad, int k_pad) {
  if (n_pad <= 0 || k_pad <= 0 || k_pad % BK) return 0;
  return (size_t)n_pad * k_pad * 4 + (size_t)n_pad * 4;
}

extern "C" int raft_conv2d_split_weight_scaled(const float* w, void* out, int n_pad, int k_pad, raft_stream_t stream) {
  RAFT_REQUIRE(w && out && n_pad > 0 && k_pad > 0 && k_pad % BK == 0, "raft_conv2d_split_weight_scaled: bad args");
  RAFT_REQUIRE((const void*)w != out && ((uintptr_t)out & 15) == 0,
               "raft_conv2d_split_weight_scaled: out must be a separate 16-byte aligned buffer");
  _Float16* o = reinterpret_cast<_Float16*>(out);
  float* inv = reinterpret_cast<float*>(reinterpret_cast<char*>(out) + (size_t)n_pad * k_pad * 4);
  hipLaunchKernelGGL(split_weight_scaled_kernel, dim3((unsigned)n_pad), dim3(256), 0, as_stream(stream), w, o, inv, k_pad);
  return check_launch("raft_conv2d_split_weight_scaled");
}

extern "C" int raft_conv2d_split_weight_prec(const float* w, void* out, int n_pad, int k_pad, int precision,
                                             raft_stream_t stream) {
  RAFT_REQUIRE(precision == RAFT_PREC_F16X3 || precision == RAFT_PREC_F16 || precision == RAFT_PREC_BF16,
               "raft_conv2d_split_weight_prec: precision %d has no split form", precision);
  if (precision != RAFT_PREC_BF16) return raft_conv2d_split_weight(w, out, n_pad, k_pad, stream);
  RAFT_REQUIRE(w && out && n_pad > 0 && k_pad > 0 && k_pad % BK == 0, "raft_conv2d_split_weight_prec: bad args");
  RAFT_REQUIRE((const void*)w != out, "raft_conv2d_split_weight_prec: in-place split is not supported");
  const long total = (long)n_pad * k_pad;
  hipLaunchKernelGGL(split_weight_bf16_kernel, dim3((unsigned)cdiv_l(total, 256)), dim3(256), 0, as_stream(stream), w,
                     reinterpret_cast<__bf16*>(out), total);
  return check_launch("raft_conv2d_split_weight_prec");
}

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

namespace {
// raft_conv2d's argument checks and the GEMM view of the conv
int conv_prepare(const raft_conv2d_params* pp, ConvArgs& a, HaloOperands& o) {
  RAFT_REQUIRE(pp != nullptr, "raft_conv2d: null params");
  const raft_conv2d_params& p = *pp;
  RAFT_REQUIRE(p.in0 && p.weight && p.out, "raft_conv2d: null in0/weight/out");
  RAFT_REQUIRE(((uintptr_t)p.weight_s & 15) == 0, "raft_conv2d: weight_s must be 16-byte aligned");
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
  a.p = p;
  a.M = p.batch * p.out_h * p.out_w;
  a.ctot = ctot;
  a.taps = p.kh * p.kw;
  int n_pad = 0, k_pad = 0;
  int rc = raft_conv2d_packed_shape(p.mode, p.n, p.kh, p.kw, ctot, &n_pad, &k_pad);
  if (rc) return rc;
  a.K = k_pad;
  a.cpad = round_up(ctot, BK);
  {
    const double npix_in = (double)p.batch * p.in_h * p.in_w;
    const double b0 = npix_in * p.in0_ld * 4.0, b1 = npix_in * (p.in1_c ? p.in1_ld : 0) * 4.0;
    const double bw = (double)n_pad * k_pad * 4.0;
    RAFT_REQUIRE(b0 < 2147483648.0 && b1 < 2147483648.0 && bw < 2147483648.0,
                 "raft_conv2d: an operand exceeds 2 GiB (split the batch)");
    a.in0_bytes = (unsigned)b0;
    a.in1_bytes = (unsigned)b1;
    a.w_bytes = (unsigned)bw;
  }
  if (p.mode == RAFT_CONV_VEC) {
    RAFT_REQUIRE(p.in0_c % 4 == 0 && p.in1_c % 4 == 0, "raft_conv2d VEC: channel counts must be multiples of 4");
    RAFT_REQUIRE(p.in1_c == 0 || p.in0_c % BK == 0, "raft_conv2d VEC: seg0 channels must be a multiple of 32 with seg1");
    RAFT_REQUIRE(p.in0_ld % 4 == 0 && (p.in1_c == 0 || p.in1_ld % 4 == 0), "raft_conv2d VEC: ld must be a multiple of 4");
    RAFT_REQUIRE(((uintptr_t)p.in0 & 15) == 0 && ((uintptr_t)p.in1 & 15) == 0,
                 "raft_conv2d VEC: inputs must be 16-byte aligned");
    RAFT_REQUIRE((long)p.batch * p.in_h * p.in_w < (1L << 24) && p.in0_ld < (1 << 20) && p.in1_ld < (1 << 20),
                 "raft_conv2d VEC: more than 2^24 input pixels (split the batch)");
  } else {
    RAFT_REQUIRE(k_pad <= MAX_GATHER_K && ctot < 1024 && p.kw < 1024,
                 "raft_conv2d GATHER: kh*kw*cin must be <= %d (got %d)", MAX_GATHER_K, p.kh * p.kw * ctot);
  }
  RAFT_REQUIRE(((uintptr_t)p.weight & 15) == 0, "raft_conv2d: weight must be 16-byte aligned");
  {
    // the epilogue indexes rows with 32-bit element offsets
    int ldmax = p.out_ld;
    if (p.out1) ldmax = ldmax > p.out1_ld ? ldmax : p.out1_ld;
    if (p.aux0) ldmax = ldmax > p.aux0_ld ? ldmax : p.aux0_ld;
    if (p.aux1) ldmax = ldmax > p.aux1_ld ? ldmax : p.aux1_ld;
    if (p.add0) ldmax = ldmax > p.add0_ld ? ldmax : p.add0_ld;
    RAFT_REQUIRE((long)a.M * ldmax < (1L << 30), "raft_conv2d: output rows exceed 2^30 elements (split the batch)");
  }
  switch (p.epilogue) {
    case RAFT_EPI_RESID_RELU:
      RAFT_REQUIRE(p.aux0, "raft_conv2d: RESID_RELU needs aux0");
      break;
    case RAFT_EPI_GRU_ZR:
      RAFT_REQUIRE(p.aux0 && p.out1 && p.split > 0 && p.split < p.n && p.split % 32 == 0,
                   "raft_conv2d: GRU_ZR needs aux0, out1 and split (a multiple of 32)");
      break;
    case RAFT_EPI_GRU_Q:
      RAFT_REQUIRE(p.aux0 && p.aux1, "raft_conv2d: GRU_Q needs aux0 (h) and aux1 (z)");
      break;
    case RAFT_EPI_TANH_RELU:
      RAFT_REQUIRE(p.out1 && p.split > 0 && p.split < p.n && p.split % 32 == 0,
                   "raft_conv2d: TANH_RELU needs out1 and split (a multiple of 32)");
      break;
    case RAFT_EPI_LINEAR:
    case RAFT_EPI_RELU:
    case RAFT_EPI_ADD_TO_OUT:
      break;
    default:
      return set_error(RAFT_E_INVALID, "raft_conv2d: unknown epilogue %d", p.epilogue);
  }
  RAFT_REQUIRE(p.precision == RAFT_PREC_FP32 || p.precision == RAFT_PREC_F16X3 || p.precision == RAFT_PREC_F16 ||
                   p.precision == RAFT_PREC_BF16,
               "raft_conv2d: unknown precision %d", p.precision);
  o.p = p;
  o.k_pad = k_pad;
  o.n_pad = n_pad;
  o.w_bytes = a.w_bytes;
  o.in0_bytes = a.in0_bytes;
  o.in1_bytes = a.in1_bytes;
  return 0;
}

bool small_n(const raft_conv2d_params& p) { return p.n <= 4 && p.mode == RAFT_CONV_VEC; }

// byte range [lo, hi) of an NHWC row operand: rows x ld floats
void row_range(const void* ptr, long rows, int ld, uintptr_t& lo, uintptr_t& hi) {
  lo = (uintptr_t)ptr;
  hi = lo + (uintptr_t)(rows * (long)ld * 4);
}
bool overlaps(const void* a, long ra, int lda, const void* b, long rb, int ldb) {
  if (!a || !b) return false;
  uintptr_t a0, a1, b0, b1;
  row_range(a, ra, lda, a0, a1);
  row_range(b, rb, ldb, b0, b1);
  return a0 < b1 && b0 < a1;
}
// could a row of output a (na channels per row) and a row of output b (nb) share an element?
// Same ld: only if their column ranges meet (b's first column taken modulo ld relative to a's
// rows, a wrap into the next row included); other lds: whenever their byte ranges meet.
bool columns_meet(const void* a, long ra, int lda, int na, const void* b, long rb, int ldb, int nb) {
  if (!overlaps(a, ra, lda, b, rb, ldb)) return false;
  if (lda != ldb) return true;
  const long d = ((long)((intptr_t)b - (intptr_t)a)) / 4;
  if (((intptr_t)b - (intptr_t)a) % 4) return true;
  long c = d % lda;
  if (c < 0) c += lda;  // b's first column in a's row coordinates
  return c < na || c + nb > lda;
}
// do the two convs write a common element? (a write-write race inside one launch)
bool writes_overlap(const raft_conv2d_params& x, const raft_conv2d_params& y) {
  const long rx = (long)x.batch * x.out_h * x.out_w, ry = (long)y.batch * y.out_h * y.out_w;
  // the channels each output pointer receives: out gets all n (or n - split with out1), out1 n - split
  const void* xo[2] = {x.out, x.out1};
  const int xl[2] = {x.out_ld, x.out1_ld}, xn[2] = {x.n, x.n};
  const void* yo[2] = {y.out, y.out1};
  const int yl[2] = {y.out_ld, y.out1_ld}, yn[2] = {y.n, y.n};
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 2; ++j)
      if (xo[i] && yo[j] && columns_meet(xo[i], rx, xl[i], xn[i], yo[j], ry, yl[j], yn[j])) return true;
  return false;
}
// does conv y read anything conv x writes?
bool reads_output_of(const raft_conv2d_params& y, const raft_conv2d_params& x) {
  const long rin = (long)y.batch * y.in_h * y.in_w, rout = (long)x.batch * x.out_h * x.out_w;
  const void* outs[2] = {x.out, x.out1};
  const int olds[2] = {x.out_ld, x.out1_ld};
  const void* ins[5] = {y.in0, y.in1, y.aux0, y.aux1, y.add0};
  const int ilds[5] = {y.in0_ld, y.in1_ld, y.aux0_ld, y.aux1_ld, y.add0_ld};
  const long irows[5] = {rin, rin, (long)y.batch * y.out_h * y.out_w, (long)y.batch * y.out_h * y.out_w,
                         (long)y.batch * y.out_h * y.out_w};
  for (int i = 0; i < 2; ++i)
    for (int j = 0; j < 5; ++j)
      if (overlaps(outs[i], rout, olds[i], ins[j], irows[j], ilds[j])) return true;
  return false;
}
}  // namespace

extern "C" int raft_conv2d(const raft_conv2d_params* pp, raft_stream_t stream) {
  ConvArgs a;
  HaloOperands o;
  const int rc = conv_prepare(pp, a, o);
  if (rc) return rc;
  const raft_conv2d_params& p = *pp;
  const int n_pad = o.n_pad;
  hipStream_t s = as_stream(stream);
  if (p.n <= 4 && p.mode == RAFT_CONV_VEC) {
    if (p.n <= 2 && p.kh == 3 && p.kw == 3 && p.stride_h == 1 && p.stride_w == 1 && p.pad_h == 1 &&
        p.pad_w == 1 && p.out_h == p.in_h && p.out_w == p.in_w) {
      // 4x16 tiles while they fill the CUs; 2x16 (twice the work-groups) when not
      const long t4 = (long)p.batch * cdiv(p.out_h, 4) * cdiv(p.out_w, 16);
      static const long th4_min = [] {
        const char* e = getenv("RAFT_SN_TH4_MIN");
        return e ? atol(e) : (long)SN_TH4_MIN_TILES;
      }();
      if (t4 >= th4_min) {
        hipLaunchKernelGGL((conv_smalln3x3_kernel<2, 4>), dim3((unsigned)t4), dim3(512), 0, s, a, p.weight);
      } else {
        const long t2 = (long)p.batch * cdiv(p.out_h, 2) * cdiv(p.out_w, 16);
        hipLaunchKernelGGL((conv_smalln3x3_kernel<2, 2>), dim3((unsigned)t2), dim3(512), 0, s, a, p.weight);
      }
      return check_launch("raft_conv2d(small n 3x3)");
    }
    dim3 grid((unsigned)cdiv_l(a.M, 4));
    if (p.n <= 2)
      hipLaunchKernelGGL(conv_smalln_kernel<2>, grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL(conv_smalln_kernel<4>, grid, dim3(256), 0, s, a);
    return check_launch("raft_conv2d(small n)");
  }
  if (p.in_norm) RAFT_REQUIRE(raft_conv2d_in_norm_ok(pp), "raft_conv2d: in_norm needs a halo-kernel 3x3 conv");
  if (p.stats_part) {
    // InstanceNorm partials come from the halo / stem / GEMM epilogues (raft_conv2d_stats_slots)
    RAFT_REQUIRE(raft_conv2d_stats_slots(pp) > 0,
                 "raft_conv2d: stats_part needs a linear-epilogue conv (raft_conv2d_stats_slots > 0)");
    RAFT_REQUIRE(p.stats_ld >= p.n && ((uintptr_t)p.stats_part & 15) == 0,
                 "raft_conv2d: stats_ld >= n and a 16-B aligned stats_part");
  }
  if (p.mode == RAFT_CONV_VEC && conv_halo_launch(o, s) == 0) return check_launch("raft_conv2d(halo)");
  if (p.mode == RAFT_CONV_GATHER && conv_stem_launch(p, o.k_pad, s) == 0) return check_launch("raft_conv2d(stem)");
  a.gn = n_pad / BN;
  a.hw = p.out_h * p.out_w;
  a.tpi = p.stats_part ? cdiv(a.hw, BM) : 0;
  const long tiles = (p.stats_part ? (long)p.batch * a.tpi : (long)cdiv(a.M, BM)) * a.gn;
  RAFT_REQUIRE(tiles < (1L << 31), "raft_conv2d: too many tiles");
  dim3 grid((unsigned)tiles);
  // few tiles (fewer than ~4 per CU): two K-groups per tile give every SIMD two waves
  const bool two = tiles < 1024 && a.K / BK >= 4;
  launch_gemm(a, grid, two, s);
  return check_launch("raft_conv2d");
}

extern "C" int raft_conv2d_in_norm_ok(const raft_conv2d_params* pp) {
  ConvArgs a;
  HaloOperands o;
  if (!pp || conv_prepare(pp, a, o)) return 0;
  return pp->mode == RAFT_CONV_VEC && pp->n > 4 && conv_halo_norm_ok(o) ? 1 : 0;
}

extern "C" int raft_conv2d_halo_tile_rows(const raft_conv2d_params* pp) {
  ConvArgs a;
  HaloOperands o;
  if (!pp || conv_prepare(pp, a, o)) return 0;
  if (pp->mode != RAFT_CONV_VEC || small_n(*pp)) return 0;
  return conv_halo_tile_rows(o);
}

extern "C" int raft_conv2d_halo_tiles_per_wg(const raft_conv2d_params* pp) {
  ConvArgs a;
  HaloOperands o;
  if (!pp || conv_prepare(pp, a, o)) return 0;
  if (pp->mode != RAFT_CONV_VEC || small_n(*pp)) return 0;
  return conv_halo_tiles_per_wg(o);
}

extern "C" int raft_conv2d_stats_slots(const raft_conv2d_params* pp) {
  ConvArgs a;
  HaloOperands o;
  if (!pp || conv_prepare(pp, a, o)) return 0;
  const raft_conv2d_params& p = *pp;
  if (p.epilogue != RAFT_EPI_LINEAR || p.alpha != 1.0f || p.add0 || (p.n <= 4 && p.mode == RAFT_CONV_VEC)) return 0;
  if (p.mode == RAFT_CONV_VEC) {
    const int hs = conv_halo_stats_slots(o);
    if (hs > 0 || conv_halo_covers(o)) return hs;
    // the 64x64-tile GEMM (strided convs): two 32-row slots per tile of one image's rows
    // (RAFT_GEMM_STATS=0: none, the separate statistics pass)
    static const bool on = [] {
      const char* e = getenv("RAFT_GEMM_STATS");
      return !(e && e[0] == '0');
    }();
    return on ? 2 * cdiv(p.out_h * p.out_w, BM) : 0;
  }
  return conv_stem_stats_slots(p, o.k_pad);
}

extern "C" int raft_conv2d_pair(const raft_conv2d_params* p0, const raft_conv2d_params* p1, raft_stream_t stream) {
  ConvArgs a0, a1;
  HaloOperands o0, o1;
  int rc = conv_prepare(p0, a0, o0);
  if (rc) return rc;
  rc = conv_prepare(p1, a1, o1);
  if (rc) return rc;
  RAFT_REQUIRE(!p0->stats_part && !p1->stats_part && !p0->in_norm && !p1->in_norm,
               "raft_conv2d_pair: no stats_part / in_norm (use raft_conv2d)");
  // one launch only when neither reads what the other writes and no element is written by both
  // (otherwise: in order, as two calls)
  const bool independent = !reads_output_of(*p1, *p0) && !reads_output_of(*p0, *p1) && !writes_overlap(*p0, *p1);
  if (independent && !small_n(*p0) && !small_n(*p1) && conv_halo_launch_pair(o0, o1, as_stream(stream)) == 0)
    return check_launch("raft_conv2d_pair(halo)");
  rc = raft_conv2d(p0, stream);
  if (rc) return rc;
  return raft_conv2d(p1, stream);
}
