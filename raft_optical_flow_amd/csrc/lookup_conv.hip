// The correlation lookup fused with the motion encoder's first two convs (gfx950):
//
//   corr = CorrBlock.__call__(coords1)                      core/corr.py:56-94
//   cor  = relu(convc1(corr))   1x1, 324 -> 256             core/update.py:185,202
//   flo  = relu(convf1(flow))   7x7, 2 -> 128               core/update.py:186,205
//
// in ONE launch, with the 324-channel correlation rows never leaving the CU: a
// work-group owns a 2x16 tile of query pixels, gathers their windows from the
// tiled pyramid (the lookup of corr_pyramid.hip, four pixels per wave), writes
// the interpolated taps split into f16 hi | lo straight into an LDS A operand
// (32 rows x 352 K), and contracts it with convc1's weight on MFMA — the weight
// read straight from L2 into registers in MFMA-fragment order (no LDS ring: each
// of the 8 waves owns 32 of the 256 output channels, so no two waves read the
// same weight bytes).  convf1 runs on the VALU of the same work-group while the
// gather's tile loads are in flight.
//
// Before (round 2): the lookup + convf1 launch wrote 9.1 MB of correlation rows
// per iteration at B=1, and convc1 (its own halo-conv launch) read them back.
//
// Arithmetic: the taps are the lookup kernel's (the reference's grid_sample
// arithmetic); convc1 runs in the conv precision (f16x3: hi*hi + lo*hi + hi*lo,
// fp32 accumulation; f16 / bf16: one product); convf1 in exact fp32 FMAs.
#include "lookup_common.hpp"

namespace raft {
namespace {

constexpr int LC_TH = 2, LC_TW = 16, LC_M = 32;          // 2x16 query pixels per work-group
constexpr int LC_R = 4, LC_L = 4, LC_RD = 9;              // RAFT-full: radius 4, 4 levels
constexpr int LC_NTAP = LC_L * LC_RD * LC_RD;             // 324 correlation channels
constexpr int LC_KS = (LC_NTAP + 31) / 32;                // 11 K-steps of 32 (K = 352)
constexpr int LC_N = 256;                                 // convc1 outputs: 8 waves x 32
constexpr int LC_F1N = 128;                               // convf1 outputs: 8 waves x 16
constexpr int LC_F1K = 7, LC_F1KK = 49;
constexpr int LC_FPH = LC_TH + LC_F1K - 1, LC_FPW = LC_TW + LC_F1K - 1;  // 8 x 22 flow patch
constexpr int LC_PX = 4;                                  // query pixels per wave

// LDS (bytes)
constexpr int LC_A_BYTES = LC_KS * LC_M * 128;                       // A operand: 45056
constexpr int LC_W1_BYTES = LC_F1N * LC_F1KK * 2 * 4;                // convf1 weights: 50176
constexpr int LC_FL_BYTES = LC_FPH * LC_FPW * 8;                     // flow patch: 1408
constexpr int LC_PATCH_FLOATS = 16 * patch_rs<4>();                  // one pixel's window patch
constexpr int LC_PATCH_BYTES = 8 * LC_PATCH_FLOATS * 4;              // 34816
constexpr int LC_YT_BYTES = 8 * LC_PX * LC_L * LC_RD * 16;           // y-entries: 18432
constexpr int LC_OFF_W1 = LC_A_BYTES, LC_OFF_FL = LC_OFF_W1 + LC_W1_BYTES, LC_OFF_PATCH = LC_OFF_FL + LC_FL_BYTES,
              LC_OFF_YT = LC_OFF_PATCH + LC_PATCH_BYTES, LC_LDS = LC_OFF_YT + LC_YT_BYTES;
static_assert(LC_LDS <= 160 * 1024, "LDS budget");
static_assert(LC_PATCH_FLOATS >= 4 * LC_KS * 8, "the staging row fits a consumed patch");

struct LookupConvArgs {
  LookupArgs a;        // pyramid geometry, coords (NHWC), flow output, lookup range flag
  const h8* wfrag;     // convc1 weight, fragment order [KS][8][4][64] x 16 B (raft_lookup_conv_pack_weight)
  const float* bias;   // convc1 bias [256] or null
  float* out;          // convc1 output rows (relu), [B*H*W][out_ld]
  int out_ld;
  int* out_flag;       // range guard of the convc1 output (feeds the split convc2), or null
  FlowConvArgs f;      // convf1 (n = 128, k = 7)
  int tx_n, ty_n;      // pixel tiles per image row / column
  int ntiles;
};

__device__ __forceinline__ void wave_sync() {
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, void* lds, unsigned voff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, 0, 0, 0);
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
  const FlowConvArgs& f = g.f;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int tile = xcd_tile(blockIdx.x, gridDim.x);
  const int per = g.tx_n * g.ty_n;
  const int b = tile / per, sr = tile - b * per;
  const int y0 = (sr / g.tx_n) * LC_TH, x0 = (sr % g.tx_n) * LC_TW;
  const int H = a.H, W = a.W, P = H * W;

  // ---- 1. loads, in the order they are waited for ------------------------------------------
  // (a) convf1's weights -> LDS by DMA (49 KiB pieces over the 8 waves)
  {
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(f.w), (short)0,
                                                                        LC_W1_BYTES, 0x00020000);
    for (int pc = wv; pc < LC_W1_BYTES / 1024; pc += 8)
      dma16(rs, smem + LC_OFF_W1 + pc * 1024, (unsigned)(pc * 1024 + lane * 16));
  }
  __builtin_amdgcn_sched_barrier(0);
  // (b) the coords of convf1's 8x22 flow patch (zero padded), threads 0 .. 175
  const int fi = threadIdx.x;
  const int fyy = y0 - 3 + fi / LC_FPW, fxx = x0 - 3 + fi % LC_FPW;
  const bool fin = fi < LC_FPH * LC_FPW && (unsigned)fyy < (unsigned)H && (unsigned)fxx < (unsigned)W;
  f32x2 fc = {0.f, 0.f};
  if (fin) fc = *reinterpret_cast<const f32x2*>(a.coords + 2L * ((long)b * P + fyy * W + fxx));
  // (c) convc1's weight fragments of K-steps 0 and 1 (this wave's 32 output channels)
  h8 wb[3][NT];
  auto load_w = [&](int j, h8 (&dst)[NT]) {
#pragma unroll
    for (int t = 0; t < NT; ++t) dst[t] = g.wfrag[((j * 8 + wv) * 4 + t) * 64 + lane];
  };
  load_w(0, wb[0]);
  load_w(1, wb[1]);
  __builtin_amdgcn_sched_barrier(0);  // (a) .. (c) are issued before the tile loads: vmcnt(16) below
  // (d) the windows of this wave's four query pixels, every level, one 16-B load per lane each
  const int ti = lane >> 4, tj = (lane >> 2) & 3, rr = lane & 3;
  const int lrow = ti * 4 + rr;
  float px_x[LC_PX], px_y[LC_PX];
  int px_gp[LC_PX];
  bool px_ok[LC_PX];
  f32x4 v[LC_PX][LC_L];
#pragma unroll
  for (int k = 0; k < LC_PX; ++k) {
    const int m = LC_PX * wv + k;
    const int yy = y0 + (m >> 4), xx = x0 + (m & 15);
    const bool ok = yy < H && xx < W;
    const int gp = ok ? b * P + yy * W + xx : b * P;
    px_ok[k] = ok;
    px_gp[k] = gp;
    const float x = a.coords[2L * gp], y = a.coords[2L * gp + 1];
    px_x[k] = x;
    px_y[k] = y;
    const int xf = __builtin_amdgcn_readfirstlane((int)floorf(x));
    const int yf = __builtin_amdgcn_readfirstlane((int)floorf(y));
#pragma unroll
    for (int l = 0; l < LC_L; ++l) {
      const int wx0 = (xf >> l) - R, wy0 = (yf >> l) - R;
      const int tyo = wy0 >> 2, txo = wx0 >> 2;
      const int ntx = ((wx0 + WD - 1) >> 2) - txo + 1;
      const Level& lv = a.lv[l];
      // (the scalar-interval window test of corr_lookup_kernel<..., SCAL>)
      const int rlo = max(wy0, 0), rhi = min(wy0 + WD, 4 * lv.th);
      const int clo = max(txo, 0), chi = min(txo + ntx, lv.tw);
      const int rb = __builtin_amdgcn_readfirstlane(rlo - 4 * tyo), cb = __builtin_amdgcn_readfirstlane(clo - txo);
      const bool tok = ok && ((unsigned)(lrow - rb) < (unsigned)max(rhi - rlo, 0)) &&
                       ((unsigned)(tj - cb) < (unsigned)max(chi - clo, 0));
      const float* wbase = a.lbase[l] + (long)((unsigned long long)(unsigned)gp * (unsigned)lv.mapsz) +
                           ((long)tyo * lv.tw + txo) * 16;
      const __amdgpu_buffer_rsrc_t rs =
          __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wbase), (short)0, 0x7FFFFFFF, 0x00020000);
      const unsigned off = tok ? __umul24((unsigned)ti, (unsigned)(64 * lv.tw)) + 16u * (unsigned)(lane & 15)
                               : 0x80000000u;
      v[k][l] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
    }
  }

  LC_STAMP(1);
  // ---- 2. while the tiles fly: the per-axis sampling entries of the four pixels ------------
  // lane (l, ix) = (lane / 9, lane % 9), lanes 0 .. 35: x-entry ix kept in registers, y-entry
  // ix through LDS (the reference's arithmetic, see axis_entry)
  const bool col = lane < LC_L * RD;
  int lq = 0;
#pragma unroll
  for (int k = 1; k < LC_L; ++k) lq += lane >= k * RD ? 1 : 0;
  const int l = col ? lq : 0;
  const int ix = lane - l * RD;
  const f32x4 prm = a.prm[l];
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

  LC_STAMP(2);
  // ---- 3. convf1 on the VALU (weights + flow patch: the loads of (a), (b)) ------------------
  __builtin_amdgcn_s_waitcnt(0x0F70 | (LC_PX * LC_L & 15) | ((LC_PX * LC_L >> 4) << 14));  // vmcnt(16): all but the tiles
  float2* fl = reinterpret_cast<float2*>(smem + LC_OFF_FL);
  if (fi < LC_FPH * LC_FPW) {
    float2 fv = {0.f, 0.f};
    if (fin) {
      fv.x = round_operand(fc[0] - (float)fxx, f.rnd);
      fv.y = round_operand(fc[1] - (float)fyy, f.rnd);
    }
    fl[fi] = fv;
  }
  __syncthreads();  // the DMA'd weights and the flow patch are visible
  LC_STAMP(3);
  const int fh = lane >> 5, fm = lane & 31;
  const int fc0 = 16 * wv + 8 * fh;  // this lane's 8 convf1 channels
  float f1acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) f1acc[j] = 0.f;
  {
    const float* wl = reinterpret_cast<const float*>(smem + LC_OFF_W1) + (fc0 >> 5) * LC_F1KK * 2 * 32 + (fc0 & 31);
    const int fpy = fm >> 4, fpx = fm & 15;
#pragma unroll 1
    for (int dy = 0; dy < LC_F1K; ++dy) {
      const float2* row = fl + (fpy + dy) * LC_FPW + fpx;
      const float* wr = wl + dy * LC_F1K * 2 * 32;
#pragma unroll
      for (int dx = 0; dx < LC_F1K; ++dx) {
        const float2 fv = row[dx];
        const f32x4 w0a = *reinterpret_cast<const f32x4*>(wr + dx * 64);
        const f32x4 w0b = *reinterpret_cast<const f32x4*>(wr + dx * 64 + 4);
        const f32x4 w1a = *reinterpret_cast<const f32x4*>(wr + dx * 64 + 32);
        const f32x4 w1b = *reinterpret_cast<const f32x4*>(wr + dx * 64 + 36);
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f1acc[j] = fmaf(fv.x, w0a[j], f1acc[j]);
          f1acc[4 + j] = fmaf(fv.x, w0b[j], f1acc[4 + j]);
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
          f1acc[j] = fmaf(fv.y, w1a[j], f1acc[j]);
          f1acc[4 + j] = fmaf(fv.y, w1b[j], f1acc[4 + j]);
        }
      }
    }
  }

  // ---- 4. the taps of each pixel -> split rows of the A operand -----------------------------
#ifdef LC_STAMPS
  asm volatile("" ::"v"(f1acc[0]), "v"(f1acc[7]));
#endif
  LC_STAMP(4);
  __builtin_amdgcn_s_waitcnt(0x0F70);  // vmcnt(0): the tiles have landed
  LC_STAMP(5);
  float* patch = reinterpret_cast<float*>(smem + LC_OFF_PATCH) + wv * LC_PATCH_FLOATS;
  char* Abase = smem;
  bool big = false;
#pragma unroll
  for (int k = 0; k < LC_PX; ++k) {
    const int m = LC_PX * wv + k;
#pragma unroll
    for (int lv_ = 0; lv_ < LC_L; ++lv_) *reinterpret_cast<f32x4*>(&patch[pidx<4>(lrow, tj * 4, lv_)]) = v[k][lv_];
    wave_sync();
    const int4* yt = ytab + k * LC_L * RD;
    float val[RD];
    const float ex = 1.0f - xt[k];
    const int xwk = xw[k];
    // the common case: every entry of the wave is finite and on the patch
    if (__all(!col || onp[k])) {
      if (col) {
        const char* p0 = reinterpret_cast<const char*>(&patch[pidx<4>(0, xwk, l)]);
        const char* p1 = reinterpret_cast<const char*>(&patch[pidx<4>(0, xwk + 1, l)]);
        auto at = [](const char* bp, int byte) { return *reinterpret_cast<const float*>(bp + byte); };
#pragma unroll
        for (int iy = 0; iy < RD; ++iy) {
          const int4 ye = yt[l * RD + iy];
          const int ro = ye.x;
          const float ty = __int_as_float(ye.y), sS = __int_as_float(ye.z);
          const f32x2 c0 = {at(p0, ro), at(p0, ro + 4 * RS)}, c1 = {at(p1, ro), at(p1, ro + 4 * RS)};
          const f32x2 hh = __builtin_elementwise_fma(c0, (f32x2){ex, ex}, c1 * (f32x2){xt[k], xt[k]});
          val[iy] = fmaf(sS, hh.x, ty * hh.y);
        }
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
    if (col) {
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) big |= fabsf(val[iy]) > RAFT_RANGE_LIMIT;
    }
    // the pixel's 324 taps through the (consumed) patch as an fp32 row, then 8-channel
    // chunks split into f16 hi | lo quads of the A operand's K-step blocks
    wave_sync();
    if (col) {
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) patch[l * RD * RD + ix * RD + iy] = px_ok[k] ? val[iy] : 0.f;
    }
    wave_sync();
    if (lane < 4 * LC_KS) {
      const int c = 8 * lane;
      f32x4 q0 = *reinterpret_cast<const f32x4*>(patch + c);
      f32x4 q1 = *reinterpret_cast<const f32x4*>(patch + c + 4);
#pragma unroll
      for (int e = 0; e < 4; ++e) {
        q0[e] = c + e < LC_NTAP ? q0[e] : 0.f;
        q1[e] = c + 4 + e < LC_NTAP ? q1[e] : 0.f;
      }
      h8 hi, lo;
      split8<X3, BF>(q0, q1, hi, lo);
      const int j = lane >> 2, qd = lane & 3, sw = (m >> 1) & 7;
      char* row = Abase + j * (LC_M * 128) + m * 128;
      *reinterpret_cast<h8*>(row + ((qd ^ sw) << 4)) = hi;
      if constexpr (X3) *reinterpret_cast<h8*>(row + (((4 + qd) ^ sw) << 4)) = lo;
    }
    if (a.flow && lane < 2 && px_ok[k]) {
      const int p = px_gp[k] - b * P;
      const float gcoord = lane == 0 ? (float)(p % W) : (float)(p / W);
      a.flow[(long)px_gp[k] * a.flow_ld + lane] = (lane == 0 ? px_x[k] : px_y[k]) - gcoord;
    }
    wave_sync();  // the chunk reads are done before the next pixel's patch lands
  }
  if (a.range_flag && big) *a.range_flag = 1;
  LC_STAMP(6);
  __syncthreads();  // every A row is in LDS
  LC_STAMP(7);

  // ---- 5. convc1: [32 x 352] x [352 x 32] per wave on MFMA, weights from L2 ------------------
  const int m = lane & 31, h = lane >> 5;
  const int sw = (m >> 1) & 7;
  f32x16 acc = {}, accx = {};
#pragma unroll
  for (int j = 0; j < LC_KS; ++j) {
    if (j + 2 < LC_KS) load_w(j + 2, wb[(j + 2) % 3]);
    const char* row = Abase + j * (LC_M * 128) + m * 128;
    h8 ah[2], al[2];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      ah[qq] = *reinterpret_cast<const h8*>(row + (((2 * h + qq) ^ sw) << 4));
      if constexpr (X3) al[qq] = *reinterpret_cast<const h8*>(row + (((4 + 2 * h + qq) ^ sw) << 4));
    }
    const h8(&B)[NT] = wb[j % 3];
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      if constexpr (BF) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_bf16(__builtin_bit_cast(bf8, ah[qq]), __builtin_bit_cast(bf8, B[qq]),
                                                      acc, 0, 0, 0);
      } else {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], B[qq], acc, 0, 0, 0);
      }
      if constexpr (X3) {
        accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], B[2 + qq], accx, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[qq], B[qq], acc, 0, 0, 0);
      }
    }
  }
  if constexpr (X3) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += accx[r] * (1.0f / SPLIT_SCALE);
  }

#ifdef LC_STAMPS
  asm volatile("" ::"v"(acc[0]), "v"(acc[15]));
#endif
  LC_STAMP(8);
  // ---- 6. epilogues: convc1 (bias, relu) and convf1 -----------------------------------------
  {
    const int n = 32 * wv + m;
    const float bias = g.bias ? g.bias[n] : 0.f;
    bool obig = false;
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int yy = y0 + (mm >> 4), xx = x0 + (mm & 15);
      const float o = fmaxf(acc[r] + bias, 0.f);
      if (yy < H && xx < W) {
        obig |= o > RAFT_RANGE_LIMIT;
        g.out[((long)b * P + yy * W + xx) * g.out_ld + n] = o;
      }
    }
    if (g.out_flag && obig) *g.out_flag = 1;
  }
  {
    const int oy = y0 + (fm >> 4), ox = x0 + (fm & 15);
    if (oy < H && ox < W) {
      float o[8];
      bool fbig = false;
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        o[j] = fmaxf(f1acc[j] + (f.bias ? f.bias[fc0 + j] : 0.f), 0.f);
        fbig |= o[j] > RAFT_RANGE_LIMIT;
      }
      if (f.range_flag && fbig) *f.range_flag = 1;
      float* dst = f.out + ((long)b * P + oy * W + ox) * f.out_ld + fc0;
      *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
      *reinterpret_cast<f32x4*>(dst + 4) = f32x4{o[4], o[5], o[6], o[7]};
    }
  }
#ifdef LC_STAMPS
  __builtin_amdgcn_s_waitcnt(0);
  LC_STAMP(9);
  const unsigned long long lc_r1 = lc_real();
  const unsigned wid = blockIdx.x * 8 + wv;
  if (lane == 0 && wid < 16384) {
    unsigned long long* gs = g_lcstamp + wid * 16;
    gs[0] = lc_r0;
    gs[1] = lc_r1;
    for (int k = 0; k < 10; ++k) gs[2 + k] = lc_t[k];
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

extern "C" size_t raft_lookup_conv_weight_floats(int n, int cin) {
  if (n <= 0 || n % 32 || cin <= 0) return 0;
  return (size_t)((cin + 31) / 32) * (size_t)n * 32;
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
                                     float* flow_out, int flow_ld, int* range_flag, const void* c1_weight,
                                     const float* c1_bias, int c1_n, int c1_precision, float* c1_out, int c1_out_ld,
                                     int* c1_range_flag, const float* f1_weight, const float* f1_bias, int f1_n,
                                     int f1_k, int f1_precision, float* f1_out, int f1_out_ld, int* f1_range_flag,
                                     raft_stream_t stream) {
  RAFT_REQUIRE(L == LC_L && radius == LC_R, "raft_corr_lookup_conv: radius 4 and 4 levels only (got %d, %d)", radius,
               L);
  RAFT_REQUIRE(c1_n == LC_N && f1_n == LC_F1N, "raft_corr_lookup_conv: convc1 256 / convf1 128 outputs only");
  RAFT_REQUIRE(c1_precision == RAFT_PREC_F16X3 || c1_precision == RAFT_PREC_F16 || c1_precision == RAFT_PREC_BF16,
               "raft_corr_lookup_conv: convc1 precision must be F16X3, F16 or BF16 (got %d)", c1_precision);
  RAFT_REQUIRE(c1_weight && c1_out && c1_out_ld >= c1_n, "raft_corr_lookup_conv: bad convc1 arguments");
  RAFT_REQUIRE((((uintptr_t)c1_weight | (uintptr_t)coords) & 15) == 0 && ((uintptr_t)coords & 7) == 0,
               "raft_corr_lookup_conv: 16-B aligned weight / coords");
  LookupConvArgs g;
  // (the lookup's own output is never written: out = the convc1 rows, checked as a dummy)
  int rc = lookup_args(g.a, pyramid, B, H, W, L, radius, coords, 0, c1_out, LC_NTAP, 0, flow_out, flow_ld, range_flag);
  if (rc) return rc;
  rc = flowconv_args(g.f, "raft_corr_lookup_conv", B, H, W, f1_weight, f1_bias, f1_n, f1_k, f1_precision, f1_out,
                     f1_out_ld, f1_range_flag);
  if (rc) return rc;
  g.wfrag = reinterpret_cast<const h8*>(c1_weight);
  g.bias = c1_bias;
  g.out = c1_out;
  g.out_ld = c1_out_ld;
  g.out_flag = c1_range_flag;
  g.tx_n = cdiv(W, LC_TW);
  g.ty_n = cdiv(H, LC_TH);
  const long nt = (long)B * g.tx_n * g.ty_n;
  RAFT_REQUIRE(nt < (1L << 31), "raft_corr_lookup_conv: grid too large");
  g.ntiles = (int)nt;
  hipStream_t s = as_stream(stream);
  const dim3 grid((unsigned)nt);
  if (c1_precision == RAFT_PREC_F16X3)
    hipLaunchKernelGGL(lookup_conv_kernel<RAFT_PREC_F16X3>, grid, dim3(512), 0, s, g);
  else if (c1_precision == RAFT_PREC_F16)
    hipLaunchKernelGGL(lookup_conv_kernel<RAFT_PREC_F16>, grid, dim3(512), 0, s, g);
  else
    hipLaunchKernelGGL(lookup_conv_kernel<RAFT_PREC_BF16>, grid, dim3(512), 0, s, g);
  return check_launch("raft_corr_lookup_conv");
}
