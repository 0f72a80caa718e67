// Shared pieces of the all-pairs lookup kernels (corr_pyramid.hip: the lookup, the lookup +
// convf1 launch; lookup_conv.hip: the lookup fused with the motion encoder's convc1).
#pragma once

#include "conv_common.hpp"

namespace raft {

constexpr int LK_MAXL = 6;

struct Level {
  int h, w;       // valid size
  int th, tw;     // tiles
  long off;       // float offset of the level in the pyramid
  long mapsz;     // floats per query pixel (th*tw*16)
};

__host__ __device__ inline long tiled_index(int y, int x, int tw) {
  return ((long)(y >> 2) * tw + (x >> 2)) * 16 + (y & 3) * 4 + (x & 3);
}

struct LookupArgs {
  const float* pyr;
  Level lv[LK_MAXL];
  int B, H, W, L, r;
  const float* coords;
  int coords_layout;
  float* out;
  int out_ld, out_layout;
  float* flow;
  int flow_ld;
  int* range_flag;  // f16x3 range guard (raft_hip.h), or null
  // per level: W-1, H-1 and their reciprocals, rounded on the host exactly as
  // the device's correctly rounded 1.0f / x would
  float wm1[LK_MAXL], hm1[LK_MAXL], rw[LK_MAXL], rh[LK_MAXL];
  // the same per level as {W-1, 1/(W-1), H-1, 1/(H-1)}: one 16-B per-lane load (lane-varying level)
  f32x4 prm[LK_MAXL];
  // pyr + lv[l].off: each level's base, so a wave's per-level map address is one 32x32-bit
  // product and one 64-bit add on the scalar unit (the scalar unit is a co-limit at B=8)
  const float* lbase[LK_MAXL];
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

// q = a / b correctly rounded for normal operands, given rcp = RN(1/b): one
// Newton step on the residual (Markstein); avoids the div_scale/div_fixup path.
__device__ __forceinline__ float div_rn(float a, float b, float rcp) {
  const float q = a * rcp;
  const float r = fmaf(-q, b, a);
  return fmaf(r, rcp, q);
}

// One-axis sampling entry of offset d at level l.  The window's x and y
// sample positions are separable — tap (ix, iy) samples x-entry ix and
// y-entry iy — so the reference's per-tap coordinate arithmetic runs on
// 2(2r+1) entries per level instead of (2r+1)^2 taps.
//   w: i - patch origin when i and i + 1 lie on the staged patch; OFF_PATCH
//      when the float round trip moved the floor off it; NAN_POS when the
//      position is not finite (a 1-px level: W - 1 = 0)
constexpr int OFF_PATCH = -1000000;
constexpr int NAN_POS = -2000000;

// (fc = floor(c), computed by the caller: an integer shift of the wave's level-0 floor)
template <int R>
__device__ __forceinline__ void axis_entry(float c, int fc, int d, float m1, float rcp, int& w, float& t, int& i) {
  constexpr int WD = 2 * R + 2;
  const int v0 = fc - R;
  const int o = (v0 >> 2) * 4;                               // patch origin on this axis
  const int ext = (((v0 + WD - 1) >> 2) - (v0 >> 2) + 1) * 4;  // patch extent (12 or 16)
  const float X = c + (float)(d - R);
  const float g = div_rn(2.0f * X, m1, rcp) - 1.0f;
  const float u = (g + 1.0f) * (m1 * 0.5f);
  const bool fin = isfinite(u);
  const float f0 = fin ? floorf(u) : 0.f;
  t = u - f0;
  i = (int)f0;
  const int ww = i - o;
  w = !fin ? NAN_POS : (ww >= 0 && ww + 1 < ext) ? ww : OFF_PATCH;
}

// LDS patch of one wave: element (row r, column c) of level l at
// r*RSP + ((c/4)*LMAX + l)*4 + c%4 with the row stride RSP = 16*LMAX + 4 —
// levels interleaved at 16-B granularity, so a tile row of one level is one
// ds_write_b128.  The 4-float row pad makes those writes conflict-free: the 32
// lanes of a half-wave (8 rows x 4 tile columns) land on 8 distinct 16-B bank
// slots, 4 lanes each (the minimum for 512 B), where an unpadded 256-B row put
// 16 lanes on one slot.  The phase-3 reads (a level's lanes on consecutive
// columns of one row) keep distinct banks within a level.
template <int LMAX>
constexpr int patch_rs() {
  return 16 * LMAX + 4;
}
template <int LMAX>
__device__ __forceinline__ int pidx(int r, int c, int l) {
  return r * patch_rs<LMAX>() + ((c >> 2) * LMAX + l) * 4 + (c & 3);
}

struct FlowConvArgs {
  const float* w;     // [n/32][k*k][2][32] fp32 (rounded to the conv precision's operand type)
  const float* bias;  // [n] or null
  float* out;
  int out_ld;
  int n, k;           // output channels (multiple of 32), kernel size (7: RAFT's convf1)
  int rnd;            // flow operand rounding: 0 none, 1 f16, 2 bf16
  int* range_flag;    // f16x3 range guard of the output (feeds convf2), or null
  int tx, ty;         // 4x16 pixel tiles per image row / column
  int ngrp;           // n / 32
  int nblocks;        // B * ty * tx * ngrp
};

constexpr int FC_TH = 4, FC_TW = 16, FC_MAXK = 7, FC_CG = 32;  // 4x16 pixels x 32 channels per work-group
constexpr int FC_PW = FC_TW + FC_MAXK - 1, FC_PH = FC_TH + FC_MAXK - 1;  // 22 x 10 patch

__device__ __forceinline__ float round_operand(float v, int rnd) {
  if (rnd == 1) return (float)(_Float16)v;
  if (rnd == 2) return (float)(__bf16)v;
  return v;
}

// validated LookupArgs / FlowConvArgs of an entry point (0, or the error code; corr_pyramid.hip)
int lookup_args(LookupArgs& a, const float* pyramid, int B, int H, int W, int L, int radius, const float* coords,
                int coords_layout, float* out, int out_ld, int out_layout, float* flow_out, int flow_ld,
                int* range_flag);
int flowconv_args(FlowConvArgs& f, const char* who, int B, int H, int W, const float* f1_weight, const float* f1_bias,
                  int f1_n, int f1_k, int f1_precision, float* f1_out, int f1_out_ld, int* f1_range_flag);

}  // namespace raft
