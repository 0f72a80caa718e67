// The correlation lookup fused with the motion encoder's first two convs (gfx950):
//
//   corr = CorrBlock.__call__(coords1)                      core/corr.py:56-94
//   cor  = relu(convc1(corr))   1x1, 324 -> 256             core/update.py:185,202
//   flo  = relu(convf1(flow))   7x7, 2 -> 128               core/update.py:186,205
//
// in ONE launch, with the 324-channel correlation rows never leaving the CU.  A work-group
// (8 waves) owns a 2x16 tile of query pixels:
//
//   1. every wave issues the window tiles of its four pixels (all levels, one 16-B load per
//      lane each: the lookup of corr_pyramid.hip) and, behind them, the coords of convf1's
//      8x22 flow patch;
//   2. while they fly: the per-axis sampling entries (the reference's grid_sample arithmetic);
//   3. per pixel: the tiles go to a double-buffered LDS patch, the lane's nine taps are
//      interpolated and written, split into f16 hi | lo (the conv precision's operand format),
//      straight into the convc1 A operand in LDS (32 rows x 352 K); meanwhile the flow patch
//      becomes convf1's im2col A operand (32 rows x 128 K);
//   4. both convs on MFMA: each wave owns 32 of convc1's 256 outputs (and waves 0-3 32 of
//      convf1's 128); the weights come straight from L2 into registers in MFMA-fragment order
//      (raft_lookup_conv_pack_weight), so no two waves read the same weight bytes and no LDS
//      ring is needed;
//   5. epilogues: bias + relu, range guard, NHWC rows.
//
// Before (round 2): the lookup + convf1 launch wrote 9.1 MB of correlation rows per iteration
// at B=1 and convc1 (its own halo-conv launch) read them back.
//
// Arithmetic: the taps are the lookup kernel's; convc1 and convf1 run in the conv precision
// (f16x3: hi*hi + lo*hi + hi*(2048 lo)/2048, fp32 accumulation, the halo kernel's split;
// f16 / bf16: one product), as every other conv of the update block.
#include "lookup_common.hpp"

namespace raft {
namespace {

constexpr int LC_TH = 2, LC_TW = 16, LC_M = 32;          // 2x16 query pixels per work-group
constexpr int LC_R = 4, LC_L = 4, LC_RD = 9;              // RAFT-full: radius 4, 4 levels
constexpr int LC_NTAP = LC_L * LC_RD * LC_RD;             // 324 correlation channels
constexpr int LC_KS = (LC_NTAP + 31) / 32;                // 11 K-steps of 32 (K = 352)
constexpr int LC_N = 256;                                 // convc1 outputs: 8 waves x 32
constexpr int LC_F1N = 128;                               // convf1 outputs: waves 0-3 x 32
constexpr int LC_F1K = 7, LC_F1KK = 49;
constexpr int LC_F1KS = (2 * LC_F1KK + 31) / 32;          // convf1: K = 98 -> 4 K-steps (128)
constexpr int LC_FPH = LC_TH + LC_F1K - 1, LC_FPW = LC_TW + LC_F1K - 1;  // 8 x 22 flow patch
constexpr int LC_PX = 4;                                  // query pixels per wave

// LDS (bytes)
constexpr int LC_A_BYTES = LC_KS * LC_M * 128;                       // convc1 A operand: 45056
constexpr int LC_A1_BYTES = LC_F1KS * LC_M * 128;                    // convf1 A operand: 16384
constexpr int LC_FL_BYTES = LC_FPH * LC_FPW * 8;                     // flow patch: 1408
constexpr int LC_PATCH_FLOATS = 16 * patch_rs<4>();                  // one pixel's window patch
constexpr int LC_PATCH_BYTES = 8 * 2 * LC_PATCH_FLOATS * 4;          // two per wave: 69632
constexpr int LC_YT_BYTES = 8 * LC_PX * LC_L * LC_RD * 16;           // y-entries: 18432
constexpr int LC_OFF_A1 = LC_A_BYTES, LC_OFF_FL = LC_OFF_A1 + LC_A1_BYTES, LC_OFF_PATCH = LC_OFF_FL + LC_FL_BYTES,
              LC_OFF_YT = LC_OFF_PATCH + LC_PATCH_BYTES, LC_LDS = LC_OFF_YT + LC_YT_BYTES;
static_assert(LC_LDS <= 160 * 1024, "LDS budget");

struct LookupConvArgs {
  LookupArgs a;         // pyramid geometry, coords (NHWC), flow output, lookup range flag
  const h8* wfrag;      // convc1 weight, fragment order [11][8][4][64] x 16 B (raft_lookup_conv_pack_weight)
  const float* bias;    // convc1 bias [256] or null
  float* out;           // convc1 output rows (relu), [B*H*W][out_ld]
  int out_ld;
  int* out_flag;        // range guard of the convc1 output (feeds the split convc2), or null
  const h8* f1frag;     // convf1 weight, fragment order [4][4][4][64] x 16 B
  const float* f1bias;  // [128] or null
  float* f1out;
  int f1out_ld;
  int* f1flag;
  int tx_n, ty_n;       // pixel tiles per image row / column
  int span_slot;        // raft_debug_launch_span: this launch's slot of g_lc_span, or -1
};

// raft_debug_launch_span: per timed launch, the realtime (100 MHz) of its first work-group's start
// and of its last work-group's end (after its stores completed): the launch's span as it ran
constexpr int LC_SPAN_SLOTS = 256;
__device__ unsigned long long g_lc_span[2 * LC_SPAN_SLOTS];
int g_lc_span_next = -1;  // host: the next slot, -1 = off

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// f16 / bf16 hi (and f16x3 lo = f16(x - hi), unscaled, as split8) of one activation
template <bool X3, bool BF>
__device__ __forceinline__ void split1(float x, _Float16& hi, _Float16& lo) {
  if constexpr (BF) {
    hi = __builtin_bit_cast(_Float16, (__bf16)x);
  } else {
    hi = (_Float16)x;
    if constexpr (X3) lo = (_Float16)(x - (float)hi);
  }
}

#ifdef LC_STAMPS  // dev-only phase timing (tools/lc_stamps.py with a -DLC_STAMPS variant)
__device__ unsigned long long g_lcstamp[16 * 16384];
__device__ __forceinline__ unsigned long long lc_clock() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ unsigned long long lc_real() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define LC_STAMP(k) lc_t[k] = lc_clock()
#else
#define LC_STAMP(k)
#endif

template <int PREC>
__global__ __launch_bounds__(512) void lookup_conv_kernel(LookupConvArgs g) {
#ifdef LC_STAMPS
  unsigned long long lc_t[10];
  const unsigned long long lc_r0 = lc_real();
  LC_STAMP(0);
#endif
  constexpr bool X3 = PREC == RAFT_PREC_F16X3;
  constexpr bool BF = PREC == RAFT_PREC_BF16;
  constexpr int NT = X3 ? 4 : 2;  // weight fragments per K-step (hi qq0, hi qq1, lo qq0, lo qq1)
  constexpr int R = LC_R, RD = LC_RD, WD = 2 * R + 2, RS = patch_rs<4>();
  __shared__ __attribute__((aligned(1024))) char smem[LC_LDS];
  const LookupArgs& a = g.a;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  if (g.span_slot >= 0 && threadIdx.x == 0)
    atomicMin(&g_lc_span[2 * g.span_slot], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  const int per = g.tx_n * g.ty_n;
  const int b = tile / per, sr = tile - b * per;
  const int y0 = (sr / g.tx_n) * LC_TH, x0 = (sr % g.tx_n) * LC_TW;
  const int H = a.H, W = a.W, P = H * W;

  // The K stream of step 4, in registers: convc1's 11 K-steps (all waves) then convf1's 4 (waves
  // 0-3), prefetched PF steps ahead.  LC_EARLY: the first PF steps are issued here, before the coords
  // load, so that the weight bytes (the whole 360 KB split convc1 weight per work-group) stream in
  // under the coords / window-tile round trips and the taps instead of after them.
#ifndef LC_PF
#define LC_PF 3
#endif
#ifndef LC_TAPS2
#define LC_TAPS2 1
#endif
#ifndef LC_A1EARLY
#define LC_A1EARLY 0
#endif
  constexpr int PF = LC_PF;
  h8 wb[PF + 1][NT];
  auto load_w = [&](int j, h8 (&dst)[NT]) {
    const h8* wf = j < LC_KS ? g.wfrag + ((j * (LC_N / 32) + wv) * 4) * 64
                             : g.f1frag + (((j - LC_KS) * (LC_F1N / 32) + wv) * 4) * 64;
#pragma unroll
    for (int t = 0; t < NT; ++t) dst[t] = wf[t * 64 + lane];
  };

  // ---- 1. the window tiles of this wave's four query pixels (the critical path) --------------
  const int ti = lane >> 4, tj = (lane >> 2) & 3, rr = lane & 3;
  const int lrow = ti * 4 + rr;
  // per-level map geometry in registers up front (re-read from the kernel arguments inside the
  // pixel loop, each read is a scalar-cache round trip)
  int lth[LC_L], ltw[LC_L];
  unsigned lmsz[LC_L];
  const float* lbs[LC_L];
#pragma unroll
  for (int l = 0; l < LC_L; ++l) {
    lth[l] = a.lv[l].th;
    ltw[l] = a.lv[l].tw;
    lmsz[l] = (unsigned)a.lv[l].mapsz;
    lbs[l] = a.lbase[l];
  }
  float px_x[LC_PX], px_y[LC_PX];
  int px_gp[LC_PX];
  bool px_ok[LC_PX];
  // the four pixels' coords, every load issued before the first is used (uniform: scalar loads)
#pragma unroll
  for (int k = 0; k < LC_PX; ++k) {
    const int mk = LC_PX * wv + k;
    const int yy = y0 + (mk >> 4), xx = x0 + (mk & 15);
    const bool ok = yy < H && xx < W;
    px_ok[k] = ok;
    px_gp[k] = ok ? b * P + yy * W + xx : b * P;
  }
  {
    // one round trip: lane k < 4 loads pixel k's x and y (two 4-B loads), then lane reads
    int gk = px_gp[0];
#pragma unroll
    for (int k = 1; k < LC_PX; ++k) gk = (lane & 3) == k ? px_gp[k] : gk;
    const float cx = a.coords[2L * gk], cy = a.coords[2L * gk + 1];
#ifdef LC_EARLY  // (behind the coords load: its wait leaves the weight loads in flight)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < PF; ++j) load_w(j, wb[j]);
    __builtin_amdgcn_sched_barrier(0);
#endif
#pragma unroll
    for (int k = 0; k < LC_PX; ++k) {
      px_x[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cx), k));
      px_y[k] = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(cy), k));
    }
  }
#ifdef LC_STAMPS
  asm volatile("" ::"v"(px_x[0]), "v"(px_y[LC_PX - 1]));
  LC_STAMP(7);  // the coords have arrived
#endif
  // the small loads the waits below need before the tiles (loads return in order):
  // this lane's level constants, the coords of convf1's 8x22 flow patch (threads 0 .. 175), the biases
  const bool col = lane < LC_L * RD;
  int lq = 0;
#pragma unroll
  for (int k = 1; k < LC_L; ++k) lq += lane >= k * RD ? 1 : 0;
  const int l = col ? lq : 0;
  const int ix = lane - l * RD;
  const f32x4 prm = a.prm[l];
  const int fi = threadIdx.x;
  const int fyy = y0 - 3 + fi / LC_FPW, fxx = x0 - 3 + fi % LC_FPW;
  const bool fin = fi < LC_FPH * LC_FPW && (unsigned)fyy < (unsigned)H && (unsigned)fxx < (unsigned)W;
  f32x2 fc = {0.f, 0.f};
  if (fin) fc = *reinterpret_cast<const f32x2*>(a.coords + 2L * ((long)b * P + fyy * W + fxx));
  const int m = lane & 31, h = lane >> 5;
  const float c1b = g.bias ? g.bias[32 * wv + m] : 0.f;
  const float f1b = (wv < 4 && g.f1bias) ? g.f1bias[32 * wv + m] : 0.f;
  // (their waits here, behind the coords' round trip: after the window loads the compiler, which
  // cannot count the loads of the two window paths below as equal, would wait for all of them)
#ifndef LC_EARLYWAIT
#define LC_EARLYWAIT 1
#endif
  if constexpr (LC_EARLYWAIT != 0) asm volatile("" ::"v"(prm), "v"(c1b), "v"(f1b), "v"(fc));

  __builtin_amdgcn_sched_barrier(0);
  f32x4 v[LC_PX][LC_L];
  // Every level's maps within 2^31 bytes (uniform): one buffer resource per level and 32-bit byte
  // offsets, the window test per lane on the VALU.  Per (pixel, level) the scalar unit then computes
  // only the window origin and one product (~12 SALU instead of ~46 with a 64-bit base and a resource
  // per window: the scalar unit, shared by the CU's 8 waves, was the tile-issue phase's limit).
#ifndef LC_OFF32
#define LC_OFF32 1
#endif
#ifndef LC_TAB
#define LC_TAB 1
#endif
  bool off32 = LC_OFF32 != 0;
  const unsigned nmaps = (unsigned)(a.B * P);
#pragma unroll
  for (int l = 0; l < LC_L; ++l) off32 &= (unsigned long long)nmaps * lmsz[l] * 4ull < 0x7FFFFFF0ull;
  if (off32) {
    __amdgpu_buffer_rsrc_t rsl[LC_L];
    unsigned lano[LC_L], lmsz4[LC_L];  // the lane's byte offset in a window at its origin; map bytes
#pragma unroll
    for (int l = 0; l < LC_L; ++l) {
      rsl[l] = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(lbs[l]), (short)0, (int)(nmaps * lmsz[l] * 4u),
                                                 0x00020000);
      lano[l] = __umul24((unsigned)ti, (unsigned)(64 * ltw[l])) + 16u * (unsigned)(lane & 15);
      lmsz4[l] = lmsz[l] * 4u;
    }
#if LC_TAB
    // The 16 (pixel, level) windows' parameters computed once, window (k, l) on lane 4k + l, on the VALU,
    // and read back per load (3 v_readlane): the window's origin offset and its row / tile-column
    // intervals clipped to the map (relative to the lane's row / column in the window, 16 + 16 bits).
    // The per-load scalar chain (~19 SALU on the unit the CU's 8 waves share) becomes ~4.
    int t_sb, t_row, t_col;
    {
      const int ik = (lane >> 2) & 3, il = lane & 3;
      float fx = px_x[0], fy = px_y[0];
      int gpk = px_gp[0];
      bool okk = px_ok[0];
#pragma unroll
      for (int k = 1; k < LC_PX; ++k) {
        fx = ik == k ? px_x[k] : fx;
        fy = ik == k ? px_y[k] : fy;
        gpk = ik == k ? px_gp[k] : gpk;
        okk = ik == k ? px_ok[k] : okk;
      }
      int thl = lth[0], twl = ltw[0];
      unsigned msl = lmsz4[0];
#pragma unroll
      for (int l = 1; l < LC_L; ++l) {
        thl = il == l ? lth[l] : thl;
        twl = il == l ? ltw[l] : twl;
        msl = il == l ? lmsz4[l] : msl;
      }
      const int wx0 = ((int)floorf(fx) >> il) - R, wy0 = ((int)floorf(fy) >> il) - R;
      const int tyo = wy0 >> 2, txo = wx0 >> 2;
      const int ntx = ((wx0 + WD - 1) >> 2) - txo + 1;
      const int rlo = max(wy0, 0), rhi = min(wy0 + WD, 4 * thl);
      const int clo = max(txo, 0), chi = min(txo + ntx, twl);
      const int rn = okk ? max(rhi - rlo, 0) : 0, cn = max(chi - clo, 0);
      t_sb = (int)((unsigned)gpk * msl + (unsigned)(tyo * twl + txo) * 64u);
      t_row = ((rlo - 4 * tyo) & 0xFFFF) | (rn << 16);
      t_col = ((clo - txo) & 0xFFFF) | (cn << 16);
    }
#pragma unroll
    for (int k = 0; k < LC_PX; ++k) {
#pragma unroll
      for (int l = 0; l < LC_L; ++l) {
        const unsigned sb = (unsigned)__builtin_amdgcn_readlane(t_sb, 4 * k + l);
        const int rp = __builtin_amdgcn_readlane(t_row, 4 * k + l), cp = __builtin_amdgcn_readlane(t_col, 4 * k + l);
        // inside the window and the map (rows [rlo, rhi), tile columns [clo, chi)), or no access
        const bool tok = ((unsigned)(lrow - (rp & 0xFFFF)) < (unsigned)(rp >> 16)) &
                         ((unsigned)(tj - (cp & 0xFFFF)) < (unsigned)(cp >> 16));
        unsigned offv = sb + lano[l];
        asm volatile("" : "+v"(offv));  // (computed for every lane: a select, not a branch around it)
        const unsigned off = tok ? offv : 0x80000000u;
        v[k][l] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsl[l], off, 0, 0));
      }
    }
#else
#pragma unroll
    for (int k = 0; k < LC_PX; ++k) {
      const unsigned gp = (unsigned)px_gp[k];
      const int xf = __builtin_amdgcn_readfirstlane((int)floorf(px_x[k]));
      const int yf = __builtin_amdgcn_readfirstlane((int)floorf(px_y[k]));
#pragma unroll
      for (int l = 0; l < LC_L; ++l) {
        const int wx0 = (xf >> l) - R, wy0 = (yf >> l) - R;
        const int tyo = wy0 >> 2, txo = wx0 >> 2;
        const int ntx = ((wx0 + WD - 1) >> 2) - txo + 1;
        // map row / tile column this lane reads; inside the window and the map, or no access (tests
        // combined bitwise and the offset selected: no branch around the load)
        const int rowm = 4 * tyo + lrow, colt = txo + tj;
        const bool tok = px_ok[k] & ((unsigned)(rowm - wy0) < (unsigned)WD) & ((unsigned)rowm < (unsigned)(4 * lth[l])) &
                         ((unsigned)tj < (unsigned)ntx) & ((unsigned)colt < (unsigned)ltw[l]);
        const unsigned sb = gp * lmsz4[l] + (unsigned)(tyo * ltw[l] + txo) * 64u;
        unsigned offv = sb + lano[l];
        asm volatile("" : "+v"(offv));  // (computed for every lane: a select, not a branch around it)
        const unsigned off = tok ? offv : 0x80000000u;
        v[k][l] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rsl[l], off, 0, 0));
      }
    }
#endif
  } else {
#if LC_TAB
    // (pyramids past 2^31 bytes per level, e.g. config 5: 4.2 GB of level 0) the same table with each
    // window's 64-bit base address instead of the 32-bit offset (4 v_readlane per load, a resource per
    // window as before)
    int t_lo, t_hi, t_row, t_col;
    {
      const int ik = (lane >> 2) & 3, il = lane & 3;
      float fx = px_x[0], fy = px_y[0];
      int gpk = px_gp[0];
      bool okk = px_ok[0];
#pragma unroll
      for (int k = 1; k < LC_PX; ++k) {
        fx = ik == k ? px_x[k] : fx;
        fy = ik == k ? px_y[k] : fy;
        gpk = ik == k ? px_gp[k] : gpk;
        okk = ik == k ? px_ok[k] : okk;
      }
      int thl = lth[0], twl = ltw[0];
      unsigned msl = lmsz[0];
      const float* bsl = lbs[0];
#pragma unroll
      for (int l = 1; l < LC_L; ++l) {
        thl = il == l ? lth[l] : thl;
        twl = il == l ? ltw[l] : twl;
        msl = il == l ? lmsz[l] : msl;
        bsl = il == l ? lbs[l] : bsl;
      }
      const int wx0 = ((int)floorf(fx) >> il) - R, wy0 = ((int)floorf(fy) >> il) - R;
      const int tyo = wy0 >> 2, txo = wx0 >> 2;
      const int ntx = ((wx0 + WD - 1) >> 2) - txo + 1;
      const int rlo = max(wy0, 0), rhi = min(wy0 + WD, 4 * thl);
      const int clo = max(txo, 0), chi = min(txo + ntx, twl);
      const int rn = okk ? max(rhi - rlo, 0) : 0, cn = max(chi - clo, 0);
      const float* wbase = bsl + (long)((unsigned long long)(unsigned)gpk * msl) + ((long)tyo * twl + txo) * 16;
      const unsigned long long wa = reinterpret_cast<unsigned long long>(wbase);
      t_lo = (int)(unsigned)wa;
      t_hi = (int)(unsigned)(wa >> 32);
      t_row = ((rlo - 4 * tyo) & 0xFFFF) | (rn << 16);
      t_col = ((clo - txo) & 0xFFFF) | (cn << 16);
    }
#pragma unroll
    for (int k = 0; k < LC_PX; ++k) {
#pragma unroll
      for (int l = 0; l < LC_L; ++l) {
        const unsigned lo = (unsigned)__builtin_amdgcn_readlane(t_lo, 4 * k + l);
        const unsigned hi = (unsigned)__builtin_amdgcn_readlane(t_hi, 4 * k + l);
        const int rp = __builtin_amdgcn_readlane(t_row, 4 * k + l), cp = __builtin_amdgcn_readlane(t_col, 4 * k + l);
        const bool tok = ((unsigned)(lrow - (rp & 0xFFFF)) < (unsigned)(rp >> 16)) &
                         ((unsigned)(tj - (cp & 0xFFFF)) < (unsigned)(cp >> 16));
        const float* wbase = reinterpret_cast<const float*>(((unsigned long long)hi << 32) | lo);
        const __amdgpu_buffer_rsrc_t rs =
            __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wbase), (short)0, 0x7FFFFFFF, 0x00020000);
        unsigned offv = __umul24((unsigned)ti, (unsigned)(64 * ltw[l])) + 16u * (unsigned)(lane & 15);
        asm volatile("" : "+v"(offv));
        const unsigned off = tok ? offv : 0x80000000u;
        v[k][l] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
      }
    }
#else
#pragma unroll
  for (int k = 0; k < LC_PX; ++k) {
    const bool ok = px_ok[k];
    const int gp = px_gp[k];
    const int xf = __builtin_amdgcn_readfirstlane((int)floorf(px_x[k]));
    const int yf = __builtin_amdgcn_readfirstlane((int)floorf(px_y[k]));
#pragma unroll
    for (int l = 0; l < LC_L; ++l) {
      const int wx0 = (xf >> l) - R, wy0 = (yf >> l) - R;
      const int tyo = wy0 >> 2, txo = wx0 >> 2;
      const int ntx = ((wx0 + WD - 1) >> 2) - txo + 1;
      // (the scalar-interval window test of corr_lookup_kernel<..., SCAL>)
      const int rlo = max(wy0, 0), rhi = min(wy0 + WD, 4 * lth[l]);
      const int clo = max(txo, 0), chi = min(txo + ntx, ltw[l]);
      const int rb = __builtin_amdgcn_readfirstlane(rlo - 4 * tyo), cb = __builtin_amdgcn_readfirstlane(clo - txo);
      const bool tok = ok && ((unsigned)(lrow - rb) < (unsigned)max(rhi - rlo, 0)) &&
                       ((unsigned)(tj - cb) < (unsigned)max(chi - clo, 0));
      const float* wbase = lbs[l] + (long)((unsigned long long)(unsigned)gp * lmsz[l]) + ((long)tyo * ltw[l] + txo) * 16;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wbase), (short)0, 0x7FFFFFFF, 0x00020000);
      const unsigned off = tok ? __umul24((unsigned)ti, (unsigned)(64 * ltw[l])) + 16u * (unsigned)(lane & 15)
                               : 0x80000000u;
      v[k][l] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  }
#endif
  }
  LC_STAMP(1);
  // ---- 2. while the tiles fly: the per-axis sampling entries of the four pixels ------------
  // lane (l, ix) = (lane / 9, lane % 9), lanes 0 .. 35: x-entry ix kept in registers, y-entry
  // ix through LDS (the reference's arithmetic, see axis_entry)
  int4* ytab = reinterpret_cast<int4*>(smem + LC_OFF_YT) + wv * LC_PX * LC_L * RD;
  int xw[LC_PX], xi[LC_PX];
  float xt[LC_PX];
  bool onp[LC_PX];  // this lane's x- and y-entry lie on the staged patch
#pragma unroll
  for (int k = 0; k < LC_PX; ++k) {
    const float s = __builtin_ldexpf(1.0f, -l);
    const int xf = __builtin_amdgcn_readfirstlane((int)floorf(px_x[k]));
    const int yf = __builtin_amdgcn_readfirstlane((int)floorf(px_y[k]));
    axis_entry<R>(px_x[k] * s, xf >> l, ix, prm[0], prm[1], xw[k], xt[k], xi[k]);
    int yw, yi;
    float yt;
    axis_entry<R>(px_y[k] * s, yf >> l, ix, prm[2], prm[3], yw, yt, yi);
    onp[k] = xw[k] >= 0 && yw >= 0;
    if (col) ytab[k * LC_L * RD + lane] = int4{yw >= 0 ? yw * RS * 4 : yw, __float_as_int(yt), __float_as_int(1.0f - yt), yi};
  }
  // the flow patch (coords - grid, zero padded)
  float2* fl = reinterpret_cast<float2*>(smem + LC_OFF_FL);
  if (fi < LC_FPH * LC_FPW) {
    float2 fv = {0.f, 0.f};
    if (fin) {
      fv.x = fc[0] - (float)fxx;
      fv.y = fc[1] - (float)fyy;
    }
    fl[fi] = fv;
  }
  LC_STAMP(2);
#if LC_A1EARLY
  // convf1's A operand before the taps, while the window tiles are still in flight
  __syncthreads();  // the flow patch is visible
  // convf1's im2col A operand: row mm, K = 2 (dy*7 + dx) + ci (the GATHER packing), 8 K per thread
  {
    const int mm = threadIdx.x >> 4, q = threadIdx.x & 15;
    const int py = mm >> 4, px = mm & 15;
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = 8 * q + i, t = k >> 1;
      const int dy = t / LC_F1K, dx = t - dy * LC_F1K;
      const float2 fv = fl[(py + (k < 2 * LC_F1KK ? dy : 0)) * LC_FPW + px + (k < 2 * LC_F1KK ? dx : 0)];
      e[i] = k < 2 * LC_F1KK ? ((k & 1) ? fv.y : fv.x) : 0.f;
    }
    h8 hi, lo;
    split8<X3, BF>(f32x4{e[0], e[1], e[2], e[3]}, f32x4{e[4], e[5], e[6], e[7]}, hi, lo);
    const int j = q >> 2, qd = q & 3, sw = (mm >> 1) & 7;
    char* row = smem + LC_OFF_A1 + j * (LC_M * 128) + mm * 128;
    *reinterpret_cast<h8*>(row + ((qd ^ sw) << 4)) = hi;
    if constexpr (X3) *reinterpret_cast<h8*>(row + (((4 + qd) ^ sw) << 4)) = lo;
  }
#endif

  // ---- 3. the taps of each pixel -> split rows of convc1's A operand ------------------------
  // (default: the first PF K-steps of the weight stream are issued here, behind the tiles, so they
  // land during the taps)
#ifndef LC_EARLY
#pragma unroll
  for (int j = 0; j < PF; ++j) load_w(j, wb[j]);
#endif
  char* Abase = smem;
  bool big = false;
  auto patch_of = [&](int k) {
    return reinterpret_cast<float*>(smem + LC_OFF_PATCH) + (wv * 2 + (k & 1)) * LC_PATCH_FLOATS;
  };
  // this lane's nine output channels c = l*81 + ix*9 + iy
  const int cbase = l * RD * RD + ix * RD;
  // the nine taps of pixel k from its staged patch
  auto taps = [&](int k, float (&val)[RD]) {
    const float* patch = patch_of(k);
    const int4* yt = ytab + k * LC_L * RD;
    const float ex = 1.0f - xt[k];
    const int xwk = xw[k];
    // the common case: every entry of the wave is finite and on the patch
    if (__all(!col || onp[k])) {
      if (col) {
        const char* p0 = reinterpret_cast<const char*>(&patch[pidx<4>(0, xwk, l)]);
        const char* p1 = reinterpret_cast<const char*>(&patch[pidx<4>(0, xwk + 1, l)]);
        auto at = [](const char* bp, int byte) { return *reinterpret_cast<const float*>(bp + byte); };
#ifndef LC_TAPS3
#define LC_TAPS3 1
#endif
#if LC_TAPS3 && LC_TAPS2
        // The nine y-entries first.  Where every lane's nine rows are consecutive (the common case: the float
        // round trip moved no floor), tap iy's lower row is tap iy + 1's upper row: the lane reads its two
        // columns once, RD + 1 rows each (10 LDS reads of two rows, 4 * RS bytes apart, instead of 18), and
        // each tap takes its four corners from registers -- the same values, the same arithmetic.
        int ro[RD];
        float tyv[RD];
        bool cons = true;
#pragma unroll
        for (int iy = 0; iy < RD; ++iy) {
          const int2 ye = *reinterpret_cast<const int2*>(&yt[l * RD + iy]);
          ro[iy] = ye.x;
          tyv[iy] = __int_as_float(ye.y);
        }
#pragma unroll
        for (int iy = 1; iy < RD; ++iy) cons &= ro[iy] == ro[0] + iy * (4 * RS);  // (one row: 4 * RS bytes)
        if (__all(cons)) {
          const char* q0 = p0 + ro[0];
          const char* q1 = p1 + ro[0];
          float a0[RD + 1], a1[RD + 1];
#pragma unroll
          for (int r = 0; r <= RD; ++r) {
            a0[r] = at(q0, r * (4 * RS));
            a1[r] = at(q1, r * (4 * RS));
          }
#pragma unroll
          for (int iy = 0; iy < RD; ++iy) {
            const float ty = tyv[iy], sS = 1.0f - ty;
            const f32x2 c0 = {a0[iy], a0[iy + 1]}, c1 = {a1[iy], a1[iy + 1]};
            const f32x2 hh = __builtin_elementwise_fma(c0, (f32x2){ex, ex}, c1 * (f32x2){xt[k], xt[k]});
            val[iy] = fmaf(sS, hh.x, ty * hh.y);
          }
        } else {
#pragma unroll
          for (int iy = 0; iy < RD; ++iy) {
            const float ty = tyv[iy], sS = 1.0f - ty;
            const f32x2 c0 = {at(p0, ro[iy]), at(p0, ro[iy] + 4 * RS)}, c1 = {at(p1, ro[iy]), at(p1, ro[iy] + 4 * RS)};
            const f32x2 hh = __builtin_elementwise_fma(c0, (f32x2){ex, ex}, c1 * (f32x2){xt[k], xt[k]});
            val[iy] = fmaf(sS, hh.x, ty * hh.y);
          }
        }
#else
#pragma unroll
        for (int iy = 0; iy < RD; ++iy) {
#if LC_TAPS2
          // (8 of the entry's 16 bytes: one ds_read_b64, 2 LDS cycles, instead of a b96 read's 8; 1 - ty
          // is the same fp32 subtraction axis_entry stored)
          const int2 ye = *reinterpret_cast<const int2*>(&yt[l * RD + iy]);
          const int ro = ye.x;
          const float ty = __int_as_float(ye.y), sS = 1.0f - ty;
#else
          const int4 ye = yt[l * RD + iy];
          const int ro = ye.x;
          const float ty = __int_as_float(ye.y), sS = __int_as_float(ye.z);
#endif
          const f32x2 c0 = {at(p0, ro), at(p0, ro + 4 * RS)}, c1 = {at(p1, ro), at(p1, ro + 4 * RS)};
          const f32x2 hh = __builtin_elementwise_fma(c0, (f32x2){ex, ex}, c1 * (f32x2){xt[k], xt[k]});
          val[iy] = fmaf(sS, hh.x, ty * hh.y);
        }
#ifndef LC_TAPSGB
#define LC_TAPSGB 1
#endif
#if LC_TAPSGB && LC_TAPS2
        // the nine y-entries read first, then every tap's corner pairs, then the arithmetic: one LDS round
        // trip per phase instead of one per tap (the compiler had waited after each tap's reads)
        __builtin_amdgcn_sched_group_barrier(0x100, RD, 0);
        __builtin_amdgcn_sched_group_barrier(0x100, 2 * RD, 0);
        __builtin_amdgcn_sched_group_barrier(0x002, 4 * RD, 0);
#endif
#endif  // LC_TAPS3
      }
    } else if (col) {
      unsigned deferred = 0;
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) {
        const int4 ye = yt[l * RD + iy];
        const int yw2 = ye.x;
        const float ty = __int_as_float(ye.y), sS = __int_as_float(ye.z);
        const bool on = (xwk | yw2) >= 0;
        const bool nan = xwk == NAN_POS || yw2 == NAN_POS;
        const int r0 = on ? yw2 / (4 * RS) : 0, c0 = on ? xwk : 0;
        const float vv = patch[pidx<4>(r0, c0, l)] * (sS * ex) + patch[pidx<4>(r0, c0 + 1, l)] * (sS * xt[k]) +
                         patch[pidx<4>(r0 + 1, c0, l)] * (ty * ex) + patch[pidx<4>(r0 + 1, c0 + 1, l)] * (ty * xt[k]);
        val[iy] = nan ? __builtin_nanf("") : vv;
        deferred |= (!on && !nan) ? 1u << iy : 0u;
      }
      if (deferred != 0) {
        // taps whose floor the float round trip moved off the staged patch: the four
        // corners from global memory (zeros outside the map)
        const Level& lvl = a.lv[l];
        const float* mp = a.pyr + lvl.off + (long)px_gp[k] * lvl.mapsz;
        auto at = [&](int yy, int xx) {
          return ((unsigned)yy < (unsigned)lvl.h && (unsigned)xx < (unsigned)lvl.w) ? mp[tiled_index(yy, xx, lvl.tw)]
                                                                                    : 0.f;
        };
#pragma unroll
        for (int iy = 0; iy < RD; ++iy) {
          if (!((deferred >> iy) & 1u)) continue;
          const int4 ye = yt[l * RD + iy];
          const int yi = ye.w;
          const float ty = __int_as_float(ye.y), sS = __int_as_float(ye.z);
          val[iy] = at(yi, xi[k]) * (sS * ex) + at(yi, xi[k] + 1) * (sS * xt[k]) + at(yi + 1, xi[k]) * (ty * ex) +
                    at(yi + 1, xi[k] + 1) * (ty * xt[k]);
        }
      }
    }
  };
  // pixel k's taps, split, straight into its row of the A operand (2-B writes); lanes 36 .. 63
  // write the row's zero K padding (channels 324 .. 351)
  auto write_row = [&](int k, const float (&val)[RD]) {
    const int mk = LC_PX * wv + k;
    const int sw = (mk >> 1) & 7;
#if LC_TAPS2
    // the lane's nine consecutive channels as four 4-B writes of channel pairs (c even, c + 1: one
    // f16 pair of one quad) and one 2-B write, per half: 10 LDS writes instead of 18
    if (col) {
      const int par = cbase & 1;
      float vv[RD];
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) {
        vv[iy] = px_ok[k] ? val[iy] : 0.f;
        big |= fabsf(vv[iy]) > RAFT_RANGE_LIMIT;
      }
      auto at_c = [&](int c, int half) {  // byte address of channel c's f16 in half 0 (hi) / 1 (lo)
        const int j = c >> 5, kk = c & 31;
        return Abase + j * (LC_M * 128) + mk * 128 + (((4 * half + (kk >> 3)) ^ sw) << 4) + 2 * (kk & 7);
      };
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const float a0 = par ? vv[2 * q + 1] : vv[2 * q], a1 = par ? vv[2 * q + 2] : vv[2 * q + 1];
        _Float16 h0, l0, h1, l1;
        split1<X3, BF>(a0, h0, l0);
        split1<X3, BF>(a1, h1, l1);
        const int c = cbase + 2 * q + par;  // even
        *reinterpret_cast<h2*>(at_c(c, 0)) = h2{h0, h1};
        if constexpr (X3) *reinterpret_cast<h2*>(at_c(c, 1)) = h2{l0, l1};
      }
      {
        const float a = par ? vv[0] : vv[RD - 1];
        _Float16 hs, ls;
        split1<X3, BF>(a, hs, ls);
        const int c = cbase + (par ? 0 : RD - 1);
        *reinterpret_cast<_Float16*>(at_c(c, 0)) = hs;
        if constexpr (X3) *reinterpret_cast<_Float16*>(at_c(c, 1)) = ls;
      }
    } else if (lane - LC_L * RD < 32 * LC_KS - LC_NTAP) {
#else
    if (col) {
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) {
        const float vv = px_ok[k] ? val[iy] : 0.f;
        big |= fabsf(vv) > RAFT_RANGE_LIMIT;
        const int c = cbase + iy;
        const int j = c >> 5, kk = c & 31;
        _Float16 hi, lo;
        split1<X3, BF>(vv, hi, lo);
        char* rb = Abase + j * (LC_M * 128) + mk * 128;
        *reinterpret_cast<_Float16*>(rb + (((kk >> 3) ^ sw) << 4) + 2 * (kk & 7)) = hi;
        if constexpr (X3) *reinterpret_cast<_Float16*>(rb + (((4 + (kk >> 3)) ^ sw) << 4) + 2 * (kk & 7)) = lo;
      }
    } else if (lane - LC_L * RD < 32 * LC_KS - LC_NTAP) {
#endif
      const int c = LC_NTAP + lane - LC_L * RD;
      const int j = c >> 5, kk = c & 31;
      char* rb = Abase + j * (LC_M * 128) + mk * 128;
      *reinterpret_cast<_Float16*>(rb + (((kk >> 3) ^ sw) << 4) + 2 * (kk & 7)) = (_Float16)0.f;
      if constexpr (X3) *reinterpret_cast<_Float16*>(rb + (((4 + (kk >> 3)) ^ sw) << 4) + 2 * (kk & 7)) = (_Float16)0.f;
    }
    if (a.flow && lane < 2 && px_ok[k]) {
      const int p = px_gp[k] - b * P;
      const float gcoord = lane == 0 ? (float)(p % W) : (float)(p / W);
      a.flow[(long)px_gp[k] * a.flow_ld + lane] = (lane == 0 ? px_x[k] : px_y[k]) - gcoord;
    }
  };
  // two pixels per round: both patches staged, one wave sync, both pixels' taps interleaved
#pragma unroll
  for (int k = 0; k < LC_PX; k += 2) {
#pragma unroll
    for (int lv_ = 0; lv_ < LC_L; ++lv_) {
      *reinterpret_cast<f32x4*>(&patch_of(k)[pidx<4>(lrow, tj * 4, lv_)]) = v[k][lv_];
      *reinterpret_cast<f32x4*>(&patch_of(k + 1)[pidx<4>(lrow, tj * 4, lv_)]) = v[k + 1][lv_];
    }
    wave_sync();
    float va[RD], vb[RD];
    taps(k, va);
    taps(k + 1, vb);
    write_row(k, va);
    write_row(k + 1, vb);
    wave_sync();  // (the patches are read before the next round overwrites them)
  }
  if (a.range_flag && big) *a.range_flag = 1;
  LC_STAMP(3);
#if LC_A1EARLY
  __syncthreads();  // every A row is in LDS
#else
  __syncthreads();  // the flow patch is visible
  // convf1's im2col A operand: row mm, K = 2 (dy*7 + dx) + ci (the GATHER packing), 8 K per thread
  {
    const int mm = threadIdx.x >> 4, q = threadIdx.x & 15;
    const int py = mm >> 4, px = mm & 15;
    float e[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) {
      const int k = 8 * q + i, t = k >> 1;
      const int dy = t / LC_F1K, dx = t - dy * LC_F1K;
      const float2 fv = fl[(py + (k < 2 * LC_F1KK ? dy : 0)) * LC_FPW + px + (k < 2 * LC_F1KK ? dx : 0)];
      e[i] = k < 2 * LC_F1KK ? ((k & 1) ? fv.y : fv.x) : 0.f;
    }
    h8 hi, lo;
    split8<X3, BF>(f32x4{e[0], e[1], e[2], e[3]}, f32x4{e[4], e[5], e[6], e[7]}, hi, lo);
    const int j = q >> 2, qd = q & 3, sw = (mm >> 1) & 7;
    char* row = smem + LC_OFF_A1 + j * (LC_M * 128) + mm * 128;
    *reinterpret_cast<h8*>(row + ((qd ^ sw) << 4)) = hi;
    if constexpr (X3) *reinterpret_cast<h8*>(row + (((4 + qd) ^ sw) << 4)) = lo;
  }
  __syncthreads();  // every A row is in LDS
#endif
  LC_STAMP(4);

  // ---- 4. convc1 (all waves, 32 outputs each) then convf1 (waves 0-3) on MFMA: one K stream ----
  const int sw = (m >> 1) & 7;
  auto kstep = [&](const char* A, const h8 (&B)[NT], f32x16& c, f32x16& cx) {
    const char* row = A + m * 128;
    h8 ah[2], al[2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      ah[qq] = *reinterpret_cast<const h8*>(row + (((2 * h + qq) ^ sw) << 4));
      if constexpr (X3) al[qq] = *reinterpret_cast<const h8*>(row + (((4 + 2 * h + qq) ^ sw) << 4));
    }
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      if constexpr (BF) {
        c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, ah[qq]), __builtin_bit_cast(bf8, B[qq]), c,
                                                    0, 0, 0);
      } else {
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], B[qq], c, 0, 0, 0);
      }
      if constexpr (X3) {
        cx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], B[2 + qq], cx, 0, 0, 0);
        c = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[qq], B[qq], c, 0, 0, 0);
      }
    }
  };
  f32x16 acc = {}, accx = {}, facc = {}, faccx = {};
  const bool f1w = wv < LC_F1N / 32;  // (wave-uniform)
#ifndef LC_SGB
#define LC_SGB 1
#endif
  if constexpr (LC_SGB) {
    // The K stream with its schedule pinned (one scheduling region per K-step): the weight loads of step
    // j + PF first, then the A fragments of step j + 1 from LDS one per MFMA gap beside step j's MFMAs.  Left
    // to itself the compiler sank both to just before their use (a vmcnt / lgkmcnt wait per MFMA pair: the L2
    // round trip of every weight K-step exposed).  Every statement is unconditional so a step is one basic
    // block: waves 4-7 load convf1's weight addresses of wave 3 and read its A operand without using them.
    struct AF {
      h8 ah[2], al[2];
    };
    auto read_af = [&](const char* A, AF& f) {
      const char* row = A + m * 128;
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        f.ah[qq] = *reinterpret_cast<const h8*>(row + (((2 * h + qq) ^ sw) << 4));
        if constexpr (X3) f.al[qq] = *reinterpret_cast<const h8*>(row + (((4 + 2 * h + qq) ^ sw) << 4));
      }
    };
    auto mfma_af = [&](const AF& f, const h8 (&B)[NT], f32x16& c, f32x16& cx) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        if constexpr (BF) {
          c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, f.ah[qq]), __builtin_bit_cast(bf8, B[qq]),
                                                      c, 0, 0, 0);
        } else {
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[qq], B[qq], c, 0, 0, 0);
        }
        if constexpr (X3) {
          cx = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.ah[qq], B[2 + qq], cx, 0, 0, 0);
          c = __builtin_amdgcn_mfma_f32_32x32x16_f16(f.al[qq], B[qq], c, 0, 0, 0);
        }
      }
    };
    auto load_w_any = [&](int j, h8 (&dst)[NT]) {  // (waves 4-7: convf1's steps of wave 3, unused)
      const int wq = j < LC_KS ? wv : (wv < LC_F1N / 32 ? wv : LC_F1N / 32 - 1);
      const h8* wf = j < LC_KS ? g.wfrag + ((j * (LC_N / 32) + wq) * 4) * 64
                               : g.f1frag + (((j - LC_KS) * (LC_F1N / 32) + wq) * 4) * 64;
#pragma unroll
      for (int t = 0; t < NT; ++t) dst[t] = wf[t * 64 + lane];
    };
    constexpr int NRA = X3 ? 4 : 2, NMA = X3 ? 6 : 2;
    auto groups = [&](bool loads) {
      if (loads) __builtin_amdgcn_sched_group_barrier(0x020, NT, 0);  // the weight loads first
#pragma unroll
      for (int i = 0; i < NMA; ++i) {
        if (i < NRA) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
        __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);
      }
    };
    AF af[2];
    read_af(Abase, af[0]);
#pragma unroll
    for (int j = 0; j < LC_KS; ++j) {
      __builtin_amdgcn_sched_barrier(0);
      if (j + PF < LC_KS + LC_F1KS) load_w_any(j + PF, wb[(j + PF) % (PF + 1)]);
      read_af(j + 1 < LC_KS ? Abase + (j + 1) * (LC_M * 128) : smem + LC_OFF_A1, af[(j + 1) & 1]);
      mfma_af(af[j & 1], wb[j % (PF + 1)], acc, accx);
      groups(j + PF < LC_KS + LC_F1KS);
      __builtin_amdgcn_sched_barrier(0);
    }
    if (f1w) {
#pragma unroll
      for (int j = LC_KS; j < LC_KS + LC_F1KS; ++j) {
        __builtin_amdgcn_sched_barrier(0);
        if (j + PF < LC_KS + LC_F1KS) load_w_any(j + PF, wb[(j + PF) % (PF + 1)]);
        if (j + 1 < LC_KS + LC_F1KS) read_af(smem + LC_OFF_A1 + (j + 1 - LC_KS) * (LC_M * 128), af[(j + 1) & 1]);
        mfma_af(af[j & 1], wb[j % (PF + 1)], facc, faccx);
        __builtin_amdgcn_sched_barrier(0);
      }
    }
  } else {
#pragma unroll
  for (int j = 0; j < LC_KS; ++j) {
    // (the K stream continues into convf1's steps on waves 0-3)
    if (j + PF < LC_KS || f1w) load_w(j + PF, wb[(j + PF) % (PF + 1)]);
    kstep(Abase + j * (LC_M * 128), wb[j % (PF + 1)], acc, accx);
  }
  if (f1w) {
#pragma unroll
    for (int j = LC_KS; j < LC_KS + LC_F1KS; ++j) {
      if (j + PF < LC_KS + LC_F1KS) load_w(j + PF, wb[(j + PF) % (PF + 1)]);
      kstep(smem + LC_OFF_A1 + (j - LC_KS) * (LC_M * 128), wb[j % (PF + 1)], facc, faccx);
    }
  }
  }
  if constexpr (X3) {
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      acc[r] += accx[r] * (1.0f / SPLIT_SCALE);
      facc[r] += faccx[r] * (1.0f / SPLIT_SCALE);
    }
  }
#ifdef LC_STAMPS
  asm volatile("" ::"v"(acc[0]), "v"(acc[15]), "v"(facc[0]));
#endif
  LC_STAMP(5);

  // ---- 5. epilogues: bias, relu, range guard, NHWC rows ----------------------------------------
  auto store = [&](const f32x16& c, float bias, float* out, int ld, int n, int* flag) {
    bool obig = false;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int yy = y0 + (mm >> 4), xx = x0 + (mm & 15);
      const float o = fmaxf(c[r] + bias, 0.f);
      if (yy < H && xx < W) {
        obig |= o > RAFT_RANGE_LIMIT;
        out[((long)b * P + yy * W + xx) * ld + n] = o;
      }
    }
    if (flag && obig) *flag = 1;
  };
  store(acc, c1b, g.out, g.out_ld, 32 * wv + m, g.out_flag);
  if (wv < LC_F1N / 32) store(facc, f1b, g.f1out, g.f1out_ld, 32 * wv + m, g.f1flag);
  if (g.span_slot >= 0) {  // (uniform) the work-group's end once its stores have completed
    __builtin_amdgcn_s_waitcnt(0);
    __syncthreads();
    if (threadIdx.x == 0)
      atomicMax(&g_lc_span[2 * g.span_slot + 1], (unsigned long long)__builtin_amdgcn_s_memrealtime());
  }
#ifdef LC_END_FENCE  // dev experiment: agent-scope release of the outputs before the waves exit
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
  __builtin_amdgcn_s_waitcnt(0);
#endif
#ifdef LC_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  LC_STAMP(6);
  const unsigned long long lc_r1 = lc_real();
  const unsigned wid = blockIdx.x * 8 + wv;
  if (lane == 0 && wid < 16384) {
    unsigned long long* gs = g_lcstamp + wid * 16;
    gs[0] = lc_r0;
    gs[1] = lc_r1;
    for (int k = 0; k < 7; ++k) gs[2 + k] = lc_t[k];
    gs[9] = lc_t[7];
  }
#endif
}

// fragment-order weight: [KS][N/32][4][64 lanes] x 8 halves; element (j, s, t, lane) = the split
// row n = 32 s + lane % 32, K-step j, halves lo*32 + 8 (2 (lane / 32) + qq) .. +7 with t = 2 lo + qq
__global__ void lookup_conv_pack_kernel(const h8* __restrict__ split, int k_steps, int nsub, h8* __restrict__ out) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  const int total = k_steps * nsub * 4 * 64;
  if (i >= total) return;
  const int lane = i & 63, t = (i >> 6) & 3, rest = i >> 8;
  const int s = rest % nsub, j = rest / nsub;
  const int n = 32 * s + (lane & 31), hh = lane >> 5, qq = t & 1, lo = t >> 1;
  // the split row n: k_steps blocks of 64 halves = 8 quads; quad lo*4 + 2 hh + qq
  out[i] = split[((long)n * k_steps + j) * 8 + lo * 4 + 2 * hh + qq];
}

}  // namespace
}  // namespace raft

using namespace raft;

#ifdef LC_STAMPS
extern "C" int raft_debug_lcstamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lcstamp), sizeof(unsigned long long) * (size_t)n);
}
#endif

extern "C" size_t raft_lookup_conv_weight_floats(int n, int k_pad) {
  if (n <= 0 || n % 32 || k_pad <= 0) return 0;
  return (size_t)((k_pad + 31) / 32) * (size_t)n * 32;
}

extern "C" int raft_lookup_conv_pack_weight(const void* split_weight, int n_pad, int k_pad, int n, void* out,
                                            raft_stream_t stream) {
  RAFT_REQUIRE(split_weight && out && n > 0 && n % 32 == 0 && n <= n_pad && k_pad > 0 && k_pad % 32 == 0,
               "raft_lookup_conv_pack_weight: bad arguments");
  RAFT_REQUIRE((((uintptr_t)split_weight | (uintptr_t)out) & 15) == 0, "raft_lookup_conv_pack_weight: 16-B alignment");
  const int ks = k_pad / 32, nsub = n / 32;
  const int total = ks * nsub * 256;
  hipLaunchKernelGGL(lookup_conv_pack_kernel, dim3((unsigned)cdiv(total, 256)), dim3(256), 0, as_stream(stream),
                     reinterpret_cast<const h8*>(split_weight), ks, nsub, reinterpret_cast<h8*>(out));
  return check_launch("raft_lookup_conv_pack_weight");
}

extern "C" int raft_corr_lookup_conv(const float* pyramid, int B, int H, int W, int L, int radius, const float* coords,
                                     float* flow_out, int flow_ld, int* range_flag, int precision,
                                     const void* c1_weight, const float* c1_bias, int c1_n, float* c1_out,
                                     int c1_out_ld, int* c1_range_flag, const void* f1_weight, const float* f1_bias,
                                     int f1_n, int f1_k, float* f1_out, int f1_out_ld, int* f1_range_flag,
                                     raft_stream_t stream) {
  RAFT_REQUIRE(L == LC_L && radius == LC_R, "raft_corr_lookup_conv: radius 4 and 4 levels only (got %d, %d)", radius,
               L);
  RAFT_REQUIRE(c1_n == LC_N && f1_n == LC_F1N && f1_k == LC_F1K,
               "raft_corr_lookup_conv: convc1 256 / convf1 128 outputs, convf1 7x7 only");
  RAFT_REQUIRE(precision == RAFT_PREC_F16X3 || precision == RAFT_PREC_F16 || precision == RAFT_PREC_BF16,
               "raft_corr_lookup_conv: precision must be F16X3, F16 or BF16 (got %d)", precision);
  RAFT_REQUIRE(c1_weight && c1_out && c1_out_ld >= c1_n && f1_weight && f1_out && f1_out_ld >= f1_n,
               "raft_corr_lookup_conv: bad conv arguments");
  RAFT_REQUIRE((((uintptr_t)c1_weight | (uintptr_t)f1_weight) & 15) == 0 && ((uintptr_t)coords & 7) == 0,
               "raft_corr_lookup_conv: 16-B aligned weights, 8-B aligned coords");
  LookupConvArgs g;
  // (the lookup's own output is never written: out = the convc1 rows, checked as a stand-in)
  int rc = lookup_args(g.a, pyramid, B, H, W, L, radius, coords, 0, c1_out, LC_NTAP, 0, flow_out, flow_ld, range_flag);
  if (rc) return rc;
  g.wfrag = reinterpret_cast<const h8*>(c1_weight);
  g.bias = c1_bias;
  g.out = c1_out;
  g.out_ld = c1_out_ld;
  g.out_flag = c1_range_flag;
  g.f1frag = reinterpret_cast<const h8*>(f1_weight);
  g.f1bias = f1_bias;
  g.f1out = f1_out;
  g.f1out_ld = f1_out_ld;
  g.f1flag = f1_range_flag;
  g.tx_n = cdiv(W, LC_TW);
  g.ty_n = cdiv(H, LC_TH);
  // (span timing: eager launches only, one thread, one device: a captured launch would bake its slot into
  // the graph; raft_debug_launch_span)
  hipStreamCaptureStatus cap = hipStreamCaptureStatusNone;
  const bool capturing = hipStreamIsCapturing(as_stream(stream), &cap) == hipSuccess && cap != hipStreamCaptureStatusNone;
  g.span_slot = !capturing && g_lc_span_next >= 0 && g_lc_span_next < LC_SPAN_SLOTS ? g_lc_span_next++ : -1;
  const long nt = (long)B * g.tx_n * g.ty_n;
  RAFT_REQUIRE(nt < (1L << 31), "raft_corr_lookup_conv: grid too large");
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)nt);
  if (precision == RAFT_PREC_F16X3)
    hipLaunchKernelGGL(lookup_conv_kernel<RAFT_PREC_F16X3>, grid, dim3(512), 0, s, g);
  else if (precision == RAFT_PREC_F16)
    hipLaunchKernelGGL(lookup_conv_kernel<RAFT_PREC_F16>, grid, dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL(lookup_conv_kernel<RAFT_PREC_BF16>, grid, dim3(512), 0, s, g);
  return check_launch("raft_corr_lookup_conv");
}

// launch-span timing of raft_corr_lookup_conv (include/raft_hip.h)
extern "C" int raft_debug_launch_span(int enable) {
  using namespace raft;
  unsigned long long init[2 * LC_SPAN_SLOTS];
  for (int i = 0; i < LC_SPAN_SLOTS; ++i) {
    init[2 * i] = ~0ull;
    init[2 * i + 1] = 0ull;
  }
  const hipError_t e = hipMemcpyToSymbol(HIP_SYMBOL(g_lc_span), init, sizeof(init));
  if (e != hipSuccess) return set_error((int)e, "raft_debug_launch_span: %s", hipGetErrorString(e));
  g_lc_span_next = enable ? 0 : -1;
  return 0;
}
extern "C" int raft_debug_launch_span_read(unsigned long long* host, int n) {
  using namespace raft;
  RAFT_REQUIRE(host && n > 0 && n <= 2 * LC_SPAN_SLOTS, "raft_debug_launch_span_read: bad arguments");
  const hipError_t e = hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lc_span), sizeof(unsigned long long) * (size_t)n);
  if (e != hipSuccess) return set_error((int)e, "raft_debug_launch_span_read: %s", hipGetErrorString(e));
  return 0;
}
