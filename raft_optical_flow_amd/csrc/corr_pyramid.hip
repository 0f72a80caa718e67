// All-pairs correlation pyramid and its radius-r window lookup (gfx950).
//
// Pyramid layout (include/raft_hip.h): every query pixel's level-l map is
// stored as 4x4 tiles of 16 floats (64 B = one HBM read granule), tiles
// row-major, zero in the padding beyond H_l x W_l.  A 10x10 lookup window
// then touches 3.25^2 ~ 10.6 tiles on average (~680 B) instead of ten
// row-major 40-B runs that straddle 64-B sectors (~1050 B measured): the
// lookup is a gather whose cost is the bytes it drags in.
#include "lookup_common.hpp"

namespace raft {
namespace {



// ============================================================================
// K2: all-pairs correlation volume + levels 0 and 1
//     (CorrBlock.corr core/corr.py:96-127 and CorrBlock.__init__ :25-54)
//
// GEMM per batch b: C[p1, p2] = <fmap1[p1], fmap2[p2]> / sqrt_c (a division,
// as the reference), M = N = H*W, K = C, on fp32 MFMA 32x32x2.  The N tile is
// an 8x8 block of the (h2, w2) grid: its epilogue writes 2x2 whole level-0
// tiles (two 128-B runs per query pixel) and pools the block into one whole
// level-1 tile.  Deeper levels come from pool2_tiled_kernel.
// ============================================================================
constexpr int CB_BM = 64, CB_BN = 64, CB_BK = 32, CB_LDSK = CB_BK + 4;

struct CorrBuildArgs {
  const float* f1;
  const float* f2;
  int ld, H, W, C, P;
  float sqrt_c;
  float* pyr;
  Level l0, l1;
  int has_l1;
  int nbx;  // 8x8 blocks along w2
  int nt;   // corr_build2: non-temporal level-0 / level-1 stores (a volume far past the Infinity Cache)
  // corr_build2 tile order over its 1-D grid (B x mt M tiles x ntl N tiles): groups of gm M tiles,
  // N tiles fastest within a group (nfast) or M tiles fastest; xcd: each XCD takes a contiguous
  // run of the order (blocks are dealt round-robin over the 8 XCDs)
  int B, mt, ntl, gm, nfast, xcd;
};

// X3: fp32-accurate split-f16 MFMA (RAFT_PREC_F16X3): both fmaps are split at
// staging into hi = f16(x) and lo = f16(x - hi) (unscaled; the LDS row holds
// the K-step's 32 hi then 32 lo halves, 128 B + 16 B pad) and every product is
// hi*hi + lo*hi + hi*lo on v_mfma_f32_32x32x16_f16 in three accumulators (the
// dropped lo*lo term is 2^-22 relative).  Otherwise fp32 MFMA 32x32x2.
template <bool X3>
__global__ __launch_bounds__(256) void corr_build_kernel(CorrBuildArgs a) {
  constexpr int STAGE = (CB_BM + CB_BN) * CB_LDSK;  // floats per stage (fp32 rows; x3 rows use the same 144 B)
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 1, wn = wave >> 1;
  const int b = blockIdx.z;
  const int m0 = blockIdx.x * CB_BM;
  const int by = blockIdx.y / a.nbx, bx = blockIdx.y - (blockIdx.y / a.nbx) * a.nbx;

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
    const int h2 = by * 8 + (r >> 3), w2 = bx * 8 + (r & 7);
    bv_[i] = h2 < a.H && w2 < a.W;
    brow[i] = a.f2 + ((long)b * a.P + (bv_[i] ? h2 * a.W + w2 : 0)) * a.ld + lq * 4;
  }
  // loads are unconditional (clamped addresses) and zeroed at the LDS store, so
  // the next K-step's loads stay in flight across the MFMAs (counted vmcnt)
  f32x4 ra[2], rb[2];
  bool ok_a[2], ok_b[2];
  auto gload = [&](int kc) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool cin = kc * CB_BK + lq * 4 < a.C;  // C % 4 == 0; zero-fill the K tail
      ok_a[i] = av_[i] && cin;
      ok_b[i] = bv_[i] && cin;
#ifdef CB_ABL_NOGLOAD
      ra[i] = f32x4{(float)kc, 1.f, 2.f, (float)i};
      rb[i] = f32x4{(float)i, 1.f, 2.f, (float)kc};
#else
      ra[i] = *reinterpret_cast<const f32x4*>(ok_a[i] ? arow[i] + kc * CB_BK : a.f1);
      rb[i] = *reinterpret_cast<const f32x4*>(ok_b[i] ? brow[i] + kc * CB_BK : a.f2);
#endif
    }
  };
  auto sstore = [&](int buf) {
    float* A = smem + buf * STAGE;
    float* Bt = A + CB_BM * CB_LDSK;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
    if constexpr (X3) {
      auto put = [&](float* base, int row, f32x4 v) {
        h4 hi, lo;
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const _Float16 hh = (_Float16)v[e];
          hi[e] = hh;
          lo[e] = (_Float16)(v[e] - (float)hh);
        }
        char* r = reinterpret_cast<char*>(base) + row * (CB_LDSK * 4) + lq * 8;
        *reinterpret_cast<h4*>(r) = hi;
        *reinterpret_cast<h4*>(r + 64) = lo;
      };
      put(A, lr, ok_a[0] ? ra[0] : z);
      put(A, lr + 32, ok_a[1] ? ra[1] : z);
      put(Bt, lr, ok_b[0] ? rb[0] : z);
      put(Bt, lr + 32, ok_b[1] ? rb[1] : z);
    } else {
      *reinterpret_cast<f32x4*>(A + lr * CB_LDSK + lq * 4) = ok_a[0] ? ra[0] : z;
      *reinterpret_cast<f32x4*>(A + (lr + 32) * CB_LDSK + lq * 4) = ok_a[1] ? ra[1] : z;
      *reinterpret_cast<f32x4*>(Bt + lr * CB_LDSK + lq * 4) = ok_b[0] ? rb[0] : z;
      *reinterpret_cast<f32x4*>(Bt + (lr + 32) * CB_LDSK + lq * 4) = ok_b[1] ? rb[1] : z;
    }
  };
  const int nk = cdiv(a.C, CB_BK);
  gload(0);
  sstore(0);
  __syncthreads();
  f32x16 acc = {}, acc2 = {}, acc3 = {};
  const int ao = (wm * 32 + (lane & 31)) * CB_LDSK + (lane >> 5) * 16;
  const int bo = (wn * 32 + (lane & 31)) * CB_LDSK + (lane >> 5) * 16;
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
    const bool more = kc + 1 < nk;
    if (more) gload(kc + 1);
    const float* A = smem + cur * STAGE;
    const float* Bt = A + CB_BM * CB_LDSK;
    if constexpr (X3) {
      // lane (m, h): channels 16qq + 8h .. +7 of row m: hi at byte 32qq + 16h, lo 64 bytes on
      const char* Ar = reinterpret_cast<const char*>(A) + (wm * 32 + (lane & 31)) * (CB_LDSK * 4) + (lane >> 5) * 16;
      const char* Br = reinterpret_cast<const char*>(Bt) + (wn * 32 + (lane & 31)) * (CB_LDSK * 4) + (lane >> 5) * 16;
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        const h8 xh = *reinterpret_cast<const h8*>(Ar + 32 * qq), xl = *reinterpret_cast<const h8*>(Ar + 64 + 32 * qq);
        const h8 yh = *reinterpret_cast<const h8*>(Br + 32 * qq), yl = *reinterpret_cast<const h8*>(Br + 64 + 32 * qq);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, yh, acc, 0, 0, 0);
        acc2 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, yh, acc2, 0, 0, 0);
        acc3 = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, yl, acc3, 0, 0, 0);
      }
    } else {
      f32x4 x[4], y[4];
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        x[j] = *reinterpret_cast<const f32x4*>(A + ao + 4 * j);
        y[j] = *reinterpret_cast<const f32x4*>(Bt + bo + 4 * j);
      }
#pragma unroll
      for (int s = 0; s < 16; ++s)
        acc = __builtin_amdgcn_mfma_f32_32x32x2f32(x[s >> 2][s & 3], y[s >> 2][s & 3], acc, 0, 0, 0);
    }
    if (more) sstore(cur ^ 1);
    __syncthreads();
  }
  if constexpr (X3) {
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[r] += acc2[r] + acc3[r];
  }

  // epilogue: scaled tile -> LDS T[64 p1][64 = 8 rows x 8 cols of the (h2, w2) block]
  constexpr int TLD = CB_BN + 1;
  float* T = smem;
  {
    const int n = wn * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      T[row * TLD + n] = acc[r] / a.sqrt_c;  // positions outside H x W are exact zeros
    }
  }
  __syncthreads();
  // level 0: tiles (2by + i, 2bx + j); the two tiles of a tile row are adjacent (128 B)
  for (int idx = tid; idx < CB_BM * 64; idx += 256) {
    const int row = idx >> 6, o = idx & 63;
    const int p1 = m0 + row;
    const int ti = o >> 5, tj = (o >> 4) & 1, e = o & 15;
    const int ty = 2 * by + ti, tx = 2 * bx + tj;
    if (p1 < a.P && ty < a.l0.th && tx < a.l0.tw) {
      const int n = (ti * 4 + (e >> 2)) * 8 + tj * 4 + (e & 3);
      a.pyr[a.l0.off + ((long)b * a.P + p1) * a.l0.mapsz + ((long)ty * a.l0.tw + tx) * 16 + e] = T[row * TLD + n];
    }
  }
  if (a.has_l1 && by < a.l1.th && bx < a.l1.tw) {
    // level 1: the block pooled 2x2 -> one whole 4x4 tile (zeros beyond H1 x W1)
    for (int idx = tid; idx < CB_BM * 16; idx += 256) {
      const int row = idx >> 4, e = idx & 15;
      const int p1 = m0 + row;
      if (p1 >= a.P) continue;
      const int yy = e >> 2, xx = e & 3;
      float v = 0.f;
      if (by * 4 + yy < a.l1.h && bx * 4 + xx < a.l1.w) {
        const float* t = T + row * TLD + (2 * yy) * 8 + 2 * xx;
        v = (((t[0] + t[1]) + t[8]) + t[9]) / 4.0f;  // avg_pool2d window order
      }
      a.pyr[a.l1.off + ((long)b * a.P + p1) * a.l1.mapsz + ((long)by * a.l1.tw + bx) * 16 + e] = v;
    }
  }
}

// K2 in the fp32-accurate split with 128 x 128 tiles (the forward's corr build): the same
// arithmetic as corr_build_kernel<true> per output (hi*hi, lo*hi, hi*lo accumulated per
// K-step in the same order), 8 waves of 32 x 64, so every fmap row staged serves twice the
// products (the 64 x 64 kernel moved 2 x the L2 bytes per output).  The N tile is an 8 x 16
// (h2, w2) block: per query pixel the epilogue writes two 256-B runs of level-0 tiles and one
// 128-B run of two level-1 tiles.
constexpr int CB2_BM = 128, CB2_BN = 128, CB2_TLD = CB2_BN + 4;  // 16-B aligned epilogue rows

// the (batch, M tile, N tile) of this work-group in the order CorrBuildArgs names
__device__ __forceinline__ void cb_tile(const CorrBuildArgs& a, int& b, int& mi, int& ni) {
  const long per_b = (long)a.mt * a.ntl;
  long L = blockIdx.x;
  if (a.xcd) {
    const long q = per_b * a.B / 8;
    if (L < 8 * q) L = (L & 7) * q + (L >> 3);
  }
  b = (int)(L / per_b);
  const long t = L - b * per_b;
  const long gl = (long)a.gm * a.ntl;
  const int g = (int)(t / gl), mb = g * a.gm, gsz = min(a.gm, a.mt - mb);
  const int r = (int)(t - g * gl);
  if (a.nfast) {
    mi = mb + r / a.ntl;
    ni = r - (r / a.ntl) * a.ntl;
  } else {
    mi = mb + r % gsz;
    ni = r / gsz;
  }
}

__global__ __launch_bounds__(512, 2) void corr_build2_kernel(CorrBuildArgs a) {
  constexpr int STAGE = (CB2_BM + CB2_BN) * CB_LDSK;  // floats per stage (144-B rows)
  static_assert(2 * STAGE >= CB2_BM * CB2_TLD, "the epilogue tile fits the staging area");
  static_assert(CB2_TLD % 4 == 0, "16-B aligned epilogue rows");
  __shared__ __attribute__((aligned(16))) float smem[2 * STAGE];
  const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
  const int wm = wave & 3, wn = wave >> 2;  // 32 query rows x 64 block pixels per wave
  int b, mi, ni;
  cb_tile(a, b, mi, ni);
  const int m0 = mi * CB2_BM;
  const int nbx = (a.W + 15) / 16;
  const int by = ni / nbx, bx = ni - (ni / nbx) * nbx;
  // staged rows lr, lr + 64; channel quad lq of the K-step.  The 16 lanes of a ds_write_b64 group
  // take rows R and R + 4 (row stride 36 dwords: 4 rows apart is 16 banks apart), conflict-free
  const int g16 = tid >> 4;
  const int lr = 8 * (g16 >> 2) + (g16 & 3) + 4 * ((tid >> 3) & 1), lq = tid & 7;
  const float* arow[2];
  const float* brow[2];
  bool av_[2], bv_[2];
#pragma unroll
  for (int i = 0; i < 2; ++i) {
    const int r = lr + 64 * i;
    const int p1 = m0 + r;
    av_[i] = p1 < a.P;
    arow[i] = a.f1 + ((long)b * a.P + (av_[i] ? p1 : 0)) * a.ld + lq * 4;
    const int h2 = by * 8 + (r >> 4), w2 = bx * 16 + (r & 15);
    bv_[i] = h2 < a.H && w2 < a.W;
    brow[i] = a.f2 + ((long)b * a.P + (bv_[i] ? h2 * a.W + w2 : 0)) * a.ld + lq * 4;
  }
  f32x4 ra[2], rb[2];
  bool ok_a[2], ok_b[2];
  auto gload = [&](int kc) {
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      const bool cin = kc * CB_BK + lq * 4 < a.C;  // C % 4 == 0; zero-fill the K tail
      ok_a[i] = av_[i] && cin;
      ok_b[i] = bv_[i] && cin;
#ifdef CB_ABL_NOGLOAD
      ra[i] = f32x4{(float)kc, 1.f, 2.f, (float)i};
      rb[i] = f32x4{(float)i, 1.f, 2.f, (float)kc};
#else
      ra[i] = *reinterpret_cast<const f32x4*>(ok_a[i] ? arow[i] + kc * CB_BK : a.f1);
      rb[i] = *reinterpret_cast<const f32x4*>(ok_b[i] ? brow[i] + kc * CB_BK : a.f2);
#endif
    }
  };
  auto put = [&](float* base, int row, f32x4 v) {
    h4 hi, lo;
#pragma unroll
    for (int e = 0; e < 4; ++e) {
      const _Float16 hh = (_Float16)v[e];
      hi[e] = hh;
      lo[e] = (_Float16)(v[e] - (float)hh);
    }
    char* r = reinterpret_cast<char*>(base) + row * (CB_LDSK * 4) + lq * 8;
    *reinterpret_cast<h4*>(r) = hi;
    *reinterpret_cast<h4*>(r + 64) = lo;
  };
  auto sstore = [&](int buf) {
    float* A = smem + buf * STAGE;
    float* Bt = A + CB2_BM * CB_LDSK;
    const f32x4 z = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int i = 0; i < 2; ++i) {
      put(A, lr + 64 * i, ok_a[i] ? ra[i] : z);
      put(Bt, lr + 64 * i, ok_b[i] ? rb[i] : z);
    }
  };
  const int nk = cdiv(a.C, CB_BK);
  gload(0);
  sstore(0);
  __syncthreads();
  f32x16 acc[2] = {}, accl[2] = {};  // hi*hi | lo*hi + hi*lo
  for (int kc = 0; kc < nk; ++kc) {
    const int cur = kc & 1;
#ifdef CB_ABL_NOLOAD
    const bool more = false;
#else
    const bool more = kc + 1 < nk;
#endif
    if (more) gload(kc + 1);
    const float* A = smem + cur * STAGE;
    const float* Bt = A + CB2_BM * CB_LDSK;
    const char* Ar = reinterpret_cast<const char*>(A) + (wm * 32 + (lane & 31)) * (CB_LDSK * 4) + (lane >> 5) * 16;
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      const h8 xh = *reinterpret_cast<const h8*>(Ar + 32 * qq), xl = *reinterpret_cast<const h8*>(Ar + 64 + 32 * qq);
#pragma unroll
      for (int sb = 0; sb < 2; ++sb) {
        const char* Br = reinterpret_cast<const char*>(Bt) + (wn * 64 + sb * 32 + (lane & 31)) * (CB_LDSK * 4) +
                         (lane >> 5) * 16;
        const h8 yh = *reinterpret_cast<const h8*>(Br + 32 * qq), yl = *reinterpret_cast<const h8*>(Br + 64 + 32 * qq);
#ifdef CB_ABL_NOMFMA
        acc[sb][0] += (float)xh[0] * (float)yh[0] + (float)xl[1] * (float)yl[2];
#else
        acc[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, yh, acc[sb], 0, 0, 0);
        accl[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xl, yh, accl[sb], 0, 0, 0);
        accl[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(xh, yl, accl[sb], 0, 0, 0);
#endif
      }
    }
    if (more) sstore(cur ^ 1);
    __syncthreads();
  }
  // epilogue: scaled tile -> LDS T[128 p1][128 = 8 rows x 16 cols of the (h2, w2) block]
  float* T = smem;
#pragma unroll
  for (int sb = 0; sb < 2; ++sb) {
    const int n = wn * 64 + sb * 32 + (lane & 31);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = wm * 32 + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
      T[row * CB2_TLD + n] = (acc[sb][r] + accl[sb][r]) / a.sqrt_c;
    }
  }
  __syncthreads();
  // level 0: tiles (2by + ti, 4bx + tj); the four tiles of a tile row are adjacent (256 B).
  // One 16-B store per lane: a tile row's 4 floats (e = 4 tr .. 4 tr + 3) are 4 consecutive
  // columns of the LDS tile (16-B aligned in the pyramid: offsets are multiples of 4 floats)
  for (int idx = tid; idx < CB2_BM * 32; idx += 512) {
    const int row = idx >> 5, o = (idx & 31) * 4;
    const int p1 = m0 + row;
    const int ti = o >> 6, tj = (o >> 4) & 3, e = o & 15;
    const int ty = 2 * by + ti, tx = 4 * bx + tj;
#ifdef CB_ABL_NOSTORE
    if (p1 < a.P && ty < a.l0.th && tx < a.l0.tw && p1 < 0) {
#else
    if (p1 < a.P && ty < a.l0.th && tx < a.l0.tw) {
#endif
      // one conflict-free ds_read_b128 (row stride 132 floats)
      const f32x4 v = *reinterpret_cast<const f32x4*>(T + row * CB2_TLD + (ti * 4 + (e >> 2)) * 16 + tj * 4);
      f32x4* dst = reinterpret_cast<f32x4*>(a.pyr + a.l0.off + ((long)b * a.P + p1) * a.l0.mapsz +
                                            ((long)ty * a.l0.tw + tx) * 16 + e);
      if (a.nt)
        __builtin_nontemporal_store(v, dst);
      else
        *dst = v;
    }
  }
  if (a.has_l1 && by < a.l1.th) {
    // level 1: the block pooled 2x2 -> level-1 tiles (by, 2bx + tj), zeros beyond H1 x W1;
    // one 16-B store per lane (a level-1 tile row)
    for (int idx = tid; idx < CB2_BM * 8; idx += 512) {
      const int row = idx >> 3, o = (idx & 7) * 4;
      const int p1 = m0 + row;
      const int tj = o >> 4, e = o & 15;
      const int tx1 = 2 * bx + tj;
      if (p1 >= a.P || tx1 >= a.l1.tw) continue;
#ifdef CB_ABL_NOSTORE
      if (p1 >= 0) continue;
#endif
      const int yy = e >> 2;
      f32x4 v4;
#pragma unroll
      for (int c = 0; c < 4; ++c) {
        const int xx = tj * 4 + c;
        float v = 0.f;
        if (by * 4 + yy < a.l1.h && bx * 8 + xx < a.l1.w) {
          const float* t = T + row * CB2_TLD + (2 * yy) * 16 + 2 * xx;
          const float2 u0 = *reinterpret_cast<const float2*>(t), u1 = *reinterpret_cast<const float2*>(t + 16);
          v = (((u0.x + u0.y) + u1.x) + u1.y) / 4.0f;  // avg_pool2d window order
        }
        v4[c] = v;
      }
      f32x4* dst = reinterpret_cast<f32x4*>(a.pyr + a.l1.off + ((long)b * a.P + p1) * a.l1.mapsz +
                                            ((long)by * a.l1.tw + tx1) * 16 + e);
      if (a.nt)
        __builtin_nontemporal_store(v4, dst);
      else
        *dst = v4;
    }
  }
}

// K2 on 256 x 256 tiles from pre-split maps (raft_corr_build_ws, the forward's f16x3 build).
// corr_build2 reads one LDS fragment per MFMA (its MFMA and LDS pipes both run at about half
// rate) and moves 16 B of fmap rows from L2 per output; here a work-group computes C^T for 256
// target pixels (a 16 x 16 block of (h2, w2)) x 256 query pixels: 0.5 fragment reads per MFMA
// and 8 B per output.
//   * Maps: corr_split4_kernel writes each fmap row as C/16 half-steps of 64 B (16 f16 hi | 16 f16
//     lo = f16(x - hi)), the same 4 B per channel as fp32, so a half-step of a 256-pixel tile is a
//     32 KiB LDS-DMA (buffer_load ... lds, lane-linear 16-B writes, the 16-B quads XOR-swizzled by
//     (row >> 1) & 3 on the source side: conflict-free fragment reads).  4 stages of (targets |
//     queries) = 128 KiB, issued 3 half-steps ahead by all 8 waves (4 DMAs each per half-step).
//   * Waves: wm = w & 3 takes target rows 4wm .. 4wm+3 of the block (2 MFMA blocks of 4 x 8
//     pixels), wn = w >> 2 takes 128 queries (4 blocks); per half-step 12 ds_read_b128, 24 MFMAs
//     (hi*hi, lo*hi, hi*lo of every block in ONE fp32 chain; no block's MFMAs back to back).
//   * Epilogue from registers: MFMA row m of a 4 x 8 block is target pixel (4wm + m/8, 8c + 4((m/4)&1)
//     + m%4), so lane (query, h) holds a whole 4x4 level-0 tile, register r = tile element r: four
//     16-B stores; the tile pools in registers to half a level-1 tile row pair, swapped with lane
//     ^32 so each lane stores one 16-B level-1 tile row.
//   * Persistent: work-group g runs units g, g + grid, ... (unit = image, query tile, target tile;
//     target tiles fastest, so the running work-groups share a query tile in L2); the DMAs run on
//     into the next unit while the last one's outputs are stored.
constexpr int CB4_T = 256;                      // targets and queries per unit
constexpr int CB4_ROW = 64;                     // bytes per (pixel, half-step) row
constexpr int CB4_STAGE = 2 * CB4_T * CB4_ROW;  // one half-step of targets | queries: 32 KiB
constexpr int CB4_NS = 4;                       // stages (3 half-steps in flight)

struct CB4Args {
  const char* s1;  // split query map  [B*P][C/16][64 B]
  const char* s2;  // split target map
  unsigned sbytes; // bytes of one split map
  int H, W, P, nh;  // nh = C / 16 half-steps
  float sqrt_c;
  float* pyr;
  Level l0, l1, l2;
  int nt;
  int qt, ttx, tt;  // query tiles per image; target tiles along w2; target tiles per image
  long units;       // B * qt * tt
  f32x4* sink;      // 4 KiB the epilogue's lanes without an output store to (every store
                    // instruction issues, so a wave's vmcnt after an epilogue is known)
};

__global__ __launch_bounds__(256) void corr_split4_kernel(const float* __restrict__ f, int ld, long npix, int C,
                                                          char* __restrict__ out) {
  const long i = (long)blockIdx.x * 256 + threadIdx.x;  // (pixel, group of 4 channels)
  const int ng = C / 4;
  if (i >= npix * ng) return;
  const long px = i / ng;
  const int g = (int)(i - px * ng);
  const f32x4 v = *reinterpret_cast<const f32x4*>(f + px * ld + 4 * g);
  h4 hi, lo;
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 h = (_Float16)v[e];
    hi[e] = h;
    lo[e] = (_Float16)(v[e] - (float)h);
  }
  char* r = out + px * (long)C * 4 + (g >> 2) * CB4_ROW + (g & 3) * 8;
  *reinterpret_cast<h4*>(r) = hi;
  *reinterpret_cast<h4*>(r + 32) = lo;
}

#ifdef CB4_STAMPS  // dev-only phase timing (tools/cb4_stamps.py with a -DCB4_STAMPS variant)
__device__ unsigned long long g_cb4stamp[8 * 8 * 1024];
__device__ __forceinline__ unsigned long long cb4_clock() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define CB4_ST(k)                       \
  do {                                  \
    const unsigned long long n_ = cb4_clock(); \
    cb4_t[k] += n_ - cb4_prev;          \
    cb4_prev = n_;                      \
  } while (0)
#else
#define CB4_ST(k)
#endif

// L2 (round 5): level 2 from registers too.  A level-2 cell is 4x4 level-0 pixels, i.e. exactly the
// lane's level-0 tile: avg_pool2d of the lane's four level-1 values in pool2_tiled_kernel's order (the
// same fp32 values it would read back), so the level-1 re-read pass (config 5: 1.05 GB) goes away.
// NW (round 5): 8 waves per work-group, one per CU (units of 256 targets x 256 queries, 4 stages of
// 32 KiB), or 4 waves (units of 256 targets x 128 queries, 3 stages of 24 KiB) with TWO work-groups per
// CU, so that one work-group's epilogue stores run under the other's MFMAs (with one work-group per
// CU its 8 waves store in lock-step and the MFMA pipe idles: stamps, the epilogue ~60 % of a wave).
// Measured (r05p) the 4-wave form pays only at one-round maps; it is an opt-in (RAFT_CB4_W4=1).
template <bool L1, bool L2 = false, int NW = 8>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void corr_build4_kernel(CB4Args a) {
  static_assert(L1 || !L2, "level 2 pools level 1");
  static_assert(NW == 8 || NW == 4, "8 or 4 waves");
  constexpr int TQ = NW == 8 ? CB4_T : CB4_T / 2;  // queries per unit
  constexpr int ROWS = CB4_T + TQ;                  // LDS rows of one half-step (targets | queries)
  constexpr int NS = NW == 8 ? CB4_NS : 3;          // stages
  constexpr int AHEAD = NS - 1;                     // half-steps in flight ahead of the one read
  constexpr int STAGE = ROWS * CB4_ROW;
  constexpr int NDMA = ROWS / 16 / NW;              // 1-KiB DMAs per wave and half-step
  constexpr int TDMA = 16 / NW;                     // ... of which target rows (k < TDMA)
#ifdef CB4_STAMPS
  unsigned long long cb4_t[6] = {}, cb4_prev = cb4_clock();
  const unsigned long long cb4_start = cb4_prev;
  int cb4_units = 0;
#endif
  // store instructions of one epilogue per wave: 2 x 4 blocks x (4 level-0 + 1 level-1 row)
  constexpr int NSTORE = 8 * (4 + (L1 ? 1 : 0)) + (L2 ? 4 : 0);
  __shared__ __attribute__((aligned(1024))) char smem[NS * STAGE];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int wm = w & 3, wn = NW == 8 ? w >> 2 : 0;
  const int m = lane & 31, h = lane >> 5;
  const long grid = gridDim.x;
  const unsigned rowb = (unsigned)a.nh * CB4_ROW;  // bytes per pixel row of a split map
  const __amdgpu_buffer_rsrc_t rq = make_rsrc(a.s1, a.sbytes), rt = make_rsrc(a.s2, a.sbytes);
  struct Unit {
    int b, q0, ty0, tx0;  // image, first query, first target row / column
  };
  auto unit_at = [&](long u) {
    Unit t;
    const long per = (long)a.qt * a.tt;
    t.b = (int)(u / per);
    const long r = u - (long)t.b * per;
    const int qi = (int)(r / a.tt), ti = (int)(r - (long)qi * a.tt);
    t.q0 = qi * TQ;
    t.ty0 = (ti / a.ttx) * 16;
    t.tx0 = (ti % a.ttx) * 16;
    return t;
  };
  // DMA k (0..NDMA-1) of this wave per half-step: instruction i = w + NW k moves LDS rows 16i .. 16i+15
  // (rows 0..255 targets, 256.. queries); lane: row 16i + lane/4, physical quad lane & 3
  unsigned voff[NDMA];
  auto set_offsets = [&](const Unit& t) {
#pragma unroll
    for (int k = 0; k < NDMA; ++k) {
      const int row = 16 * (w + NW * k) + (lane >> 2);
      const unsigned lq = (unsigned)((lane & 3) ^ ((row >> 1) & 3));
      bool ok;
      long px;
      if (k < TDMA) {  // target row R = 64 wm' + 32 c + m'
        const int R = row, mm = R & 31, c = (R >> 5) & 1;
        const int h2 = t.ty0 + 4 * (R >> 6) + (mm >> 3), w2 = t.tx0 + 8 * c + 4 * ((mm >> 2) & 1) + (mm & 3);
        ok = h2 < a.H && w2 < a.W;
        px = (long)t.b * a.P + (long)h2 * a.W + w2;
      } else {
        const int p1 = t.q0 + row - CB4_T;
        ok = p1 < a.P;
        px = (long)t.b * a.P + p1;
      }
      voff[k] = ok ? (unsigned)px * rowb + lq * 16u : OFF_INVALID;
    }
  };
  const long total = a.units;
  long u_is = blockIdx.x;  // unit of the next DMA
  int s_is = 0;            // its half-step
  long g_is = 0;           // global half-step counter of the next DMA (stage g % 4)
  if (u_is >= total) return;
  set_offsets(unit_at(u_is));
  auto issue = [&]() {  // the next half-step's DMAs (zeros past the last unit)
    const bool live = u_is < total;
    char* st = smem + (g_is % NS) * STAGE;
#pragma unroll
    for (int k = 0; k < NDMA; ++k)
      dma16(k < TDMA ? rt : rq, st + (w + NW * k) * 1024, live ? voff[k] : OFF_INVALID, (unsigned)s_is * CB4_ROW);
    ++g_is;
    if (++s_is == a.nh) {
      s_is = 0;
      u_is += grid;
      if (u_is < total) set_offsets(unit_at(u_is));
    }
  };
#pragma unroll
  for (int k = 0; k < AHEAD; ++k) issue();
  const int arow0 = wm * 64 + m, brow0 = CB4_T + wn * 128 + m;
  f32x16 acc[2][4];
#pragma unroll
  for (int c = 0; c < 2; ++c)
#pragma unroll
    for (int j = 0; j < 4; ++j) acc[c][j] = f32x16{};
  long g = 0;
  int since = AHEAD;  // half-steps since the last epilogue (AHEAD: none in flight)
  for (long u = blockIdx.x; u < total; u += grid) {
    for (int s = 0; s < a.nh; ++s, ++g, ++since) {
      // this wave's DMAs of half-step g (those of the two younger half-steps may fly; in the three
      // half-steps after an epilogue its NSTORE stores, younger than g's DMAs, may fly too)
      CB4_ST(5);  // loop overhead
      if (since <= AHEAD - 1)
        wait_vm<NDMA * (AHEAD - 1) + NSTORE>();
      else
        wait_vm<NDMA * (AHEAD - 1)>();
      CB4_ST(0);  // DMA wait
      // every wave's: stage g % NS readable, stage (g - 1) % NS free (the asm's memory clobber keeps
      // the compiler from moving this step's LDS reads above the barrier)
      asm volatile("s_barrier" ::: "memory");
      CB4_ST(1);  // barrier
      issue();  // half-step g + AHEAD
      CB4_ST(2);  // DMA issue
      const char* st = smem + (g % NS) * STAGE;
      h8 ah[2], al[2], bh[4], bl[4];
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int row = arow0 + 32 * c, sw = (row >> 1) & 3;
        ah[c] = *reinterpret_cast<const h8*>(st + row * CB4_ROW + ((h ^ sw) << 4));
        al[c] = *reinterpret_cast<const h8*>(st + row * CB4_ROW + (((2 + h) ^ sw) << 4));
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        const int row = brow0 + 32 * j, sw = (row >> 1) & 3;
        bh[j] = *reinterpret_cast<const h8*>(st + row * CB4_ROW + ((h ^ sw) << 4));
        bl[j] = *reinterpret_cast<const h8*>(st + row * CB4_ROW + (((2 + h) ^ sw) << 4));
      }
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[c][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], bh[j], acc[c][j], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[c][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[c], bh[j], acc[c][j], 0, 0, 0);
#pragma unroll
      for (int c = 0; c < 2; ++c)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[c][j] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[c], bl[j], acc[c][j], 0, 0, 0);
      CB4_ST(3);  // fragment reads + MFMAs
    }
    // ---- epilogue: level-0 tiles and level-1 rows of unit u from registers
    const Unit t = unit_at(u);
    const int ty = t.ty0 / 4 + wm;
#pragma unroll
    for (int j = 0; j < 4; ++j) {
      const int p1 = t.q0 + wn * 128 + j * 32 + m;
      const bool qok = p1 < a.P;
      const long qb = (long)t.b * a.P + (qok ? p1 : 0);
      float l2v[2];  // L2: the level-2 cells (ty, t.tx0 / 4 + 2c + h)
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const int tx = t.tx0 / 4 + 2 * c + h;
        float v[16];
#pragma unroll
        for (int r = 0; r < 16; ++r) v[r] = acc[c][j][r] / a.sqrt_c;
        {
          // the quad's four queries' tiles transposed by 16-B rows (lane q of the quad gets row q of
          // each): store i writes query 4k + i's tile, its rows from the quad's 4 lanes and the
          // adjacent tile (tx + 1) from lanes + 32, so 8 lanes fill one 128-B run (scattered 16-B
          // stores, one cache line per lane, ran the epilogue at a lane per clock)
          float rt[4][4];  // rt[e][i]: element e of row (lane & 3) of query 4k + i's tile
#pragma unroll
          for (int e = 0; e < 4; ++e) {
#pragma unroll
            for (int i = 0; i < 4; ++i) rt[e][i] = v[4 * i + e];
            quad_transpose(rt[e]);
          }
          const int qr = lane & 3;
#pragma unroll
          for (int i = 0; i < 4; ++i) {
            const int pi = t.q0 + wn * 128 + j * 32 + (m & ~3) + i;
            const bool ok = pi < a.P && ty < a.l0.th && tx < a.l0.tw;
            f32x4* dst = ok ? reinterpret_cast<f32x4*>(a.pyr + a.l0.off + ((long)t.b * a.P + pi) * a.l0.mapsz +
                                                       ((long)ty * a.l0.tw + tx) * 16) + qr
                            : a.sink + 4 * lane + i;
            const f32x4 x = {rt[0][i], rt[1][i], rt[2][i], rt[3][i]};
            if (a.nt)
              __builtin_nontemporal_store(x, dst);
            else
              *dst = x;
          }
        }
        if constexpr (L1) {
          // level-1 values (y1, x1) = (2 ty + ya, 2 tx + xb): avg_pool2d's window order, zeros past h1 x w1
          float pv[2][2];
#pragma unroll
          for (int ya = 0; ya < 2; ++ya)
#pragma unroll
            for (int xb = 0; xb < 2; ++xb) {
              const float s = ((v[8 * ya + 2 * xb] + v[8 * ya + 2 * xb + 1]) + v[8 * ya + 4 + 2 * xb]) + v[8 * ya + 4 + 2 * xb + 1];
              const bool in = 2 * ty + ya < a.l1.h && 2 * tx + xb < a.l1.w;
              pv[ya][xb] = in ? s / 4.0f : 0.f;
            }
          // lane h writes level-1 tile row 2 (ty & 1) + h: columns 0,1 from lane h = 0, 2,3 from h = 1
          const float o0 = __shfl_xor(pv[1 - h][0], 32), o1 = __shfl_xor(pv[1 - h][1], 32);
          const f32x4 row4 = h == 0 ? f32x4{pv[0][0], pv[0][1], o0, o1} : f32x4{o0, o1, pv[1][0], pv[1][1]};
          const int ty1 = ty >> 1, tx1 = tx >> 1;
          const bool ok = qok && ty1 < a.l1.th && tx1 < a.l1.tw;
          f32x4* dst = ok ? reinterpret_cast<f32x4*>(a.pyr + a.l1.off + qb * a.l1.mapsz +
                                                     ((long)ty1 * a.l1.tw + tx1) * 16 + (2 * (ty & 1) + h) * 4)
                          : a.sink + 4 * lane;
          if (a.nt)
            __builtin_nontemporal_store(row4, dst);
          else
            *dst = row4;
          if constexpr (L2) {
            const bool in2 = ty < a.l2.h && tx < a.l2.w;
            l2v[c] = in2 ? (((pv[0][0] + pv[0][1]) + pv[1][0]) + pv[1][1]) / 4.0f : 0.f;
          }
        }
      }
      if constexpr (L2) {
        // level-2 tile (ty0 / 16, tx0 / 16), row wm: columns 2c + h; lane h = 0 stores the row
        const float o0 = __shfl_xor(l2v[0], 32), o1 = __shfl_xor(l2v[1], 32);
        const int ty2 = t.ty0 >> 4, tx2 = t.tx0 >> 4;
        const bool ok = qok && h == 0 && ty2 < a.l2.th && tx2 < a.l2.tw;
        f32x4* dst = ok ? reinterpret_cast<f32x4*>(a.pyr + a.l2.off + qb * a.l2.mapsz + ((long)ty2 * a.l2.tw + tx2) * 16 +
                                                   wm * 4)
                        : a.sink + 4 * lane;
        const f32x4 row4 = {l2v[0], o0, l2v[1], o1};
        if (a.nt)
          __builtin_nontemporal_store(row4, dst);
        else
          *dst = row4;
      }
    }
#pragma unroll
    for (int c = 0; c < 2; ++c)
#pragma unroll
      for (int j = 0; j < 4; ++j) acc[c][j] = f32x16{};
    since = 0;
    CB4_ST(4);  // epilogue
#ifdef CB4_STAMPS
    ++cb4_units;
#endif
  }
  wait_vm<0>();  // (the DMAs past the last unit load zeros; nothing may land after exit)
#ifdef CB4_STAMPS
  if (lane == 0 && blockIdx.x < 1024) {
    unsigned long long* gs = g_cb4stamp + ((long)blockIdx.x * 8 + w) * 8;
    for (int k = 0; k < 6; ++k) gs[k] = cb4_t[k];
    gs[6] = cb4_clock() - cb4_start;
    gs[7] = (unsigned long long)cb4_units;
  }
#endif
}

// Level l -> l+1 2x2 average pool (floor), tiled -> tiled, zeros in the padding.
__global__ void pool2_tiled_kernel(const float* pyr, float* out_base, long n_maps, Level src,
                                   Level dst) {
  const long total = n_maps * dst.mapsz;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const long q = i / dst.mapsz;
    const int r = (int)(i - q * dst.mapsz);
    const int tile = r >> 4, e = r & 15;
    const int y = (tile / dst.tw) * 4 + (e >> 2), x = (tile % dst.tw) * 4 + (e & 3);
    float v = 0.f;
    if (y < dst.h && x < dst.w) {
      const float* m = pyr + src.off + q * src.mapsz;
      const float a0 = m[tiled_index(2 * y, 2 * x, src.tw)];
      const float a1 = m[tiled_index(2 * y, 2 * x + 1, src.tw)];
      const float a2 = m[tiled_index(2 * y + 1, 2 * x, src.tw)];
      const float a3 = m[tiled_index(2 * y + 1, 2 * x + 1, src.tw)];
      v = (((a0 + a1) + a2) + a3) / 4.0f;
    }
    out_base[dst.off + i] = v;
  }
}

// Tiled -> row-major copy of one level (API accessor CorrBlock.corr_pyramid).
__global__ void untile_kernel(const float* __restrict__ pyr, float* __restrict__ out, long n_maps, Level lv) {
  const long total = n_maps * lv.h * lv.w;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int x = i % lv.w;
    const long t = i / lv.w;
    const int y = t % lv.h;
    const long q = t / lv.h;
    out[i] = pyr[lv.off + q * lv.mapsz + tiled_index(y, x, lv.tw)];
  }
}

// ============================================================================
// K1: radius-r lookup of every level (CorrBlock.__call__ core/corr.py:56-94)
//
// One wave per query pixel.  Phase 1: per level, the <= 4x4 tiles that cover
// the (2r+2)^2 integer window around floor(coords/2^l) - r are read with one
// 16-B load per lane (lane = tile row; tiles outside the window or the map are
// skipped / zero) — all levels' loads in flight together — and staged as a
// 16x16 LDS patch.  Phase 2: each lane evaluates taps of the (2r+1)^2 x L
// output with the reference's arithmetic (offset added to the centroid, then
// bilinear_sampler's 2x/(W-1)-1 and grid_sample's (g+1)*((W-1)/2)), so corner
// indices and weights are the reference's; corners come from the LDS patch
// (or from global memory when the float round trip moved a tap's floor off
// it).  Output channel = lvl*(2r+1)^2 + ix*(2r+1) + iy, contiguous per pixel.
// ============================================================================

#ifdef LK_STAMPS  // dev-only phase timing of the lookup (tools/lookup_bench.py LKSTAMPS=1)
__device__ unsigned long long g_lkstamp[8 * 65536];
__device__ __forceinline__ unsigned long long lk_clock(bool real) {
  unsigned long long t;
  __builtin_amdgcn_s_waitcnt(0);
  __builtin_amdgcn_sched_barrier(0);
  if (real)
    asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  else
    asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#define LK_STAMP(k) const unsigned long long lk_t##k = lk_clock(false)
#else
#define LK_STAMP(k)
#endif

// ============================================================================
// The lookup and the motion encoder's first flow conv in one launch
// (core/update.py:186,205: flo = relu(convf1(flow)), a 7x7 conv of the 2-channel
// flow = coords1 - coords0).  convf1 does not read the lookup's outputs: it
// takes the flow from the same coords.  As its own GEMM launch it is K = 98 —
// a few microseconds of MFMA work behind a launch's fixed cost; here its
// work-groups (dispatched first) run on the VALU beside the memory-bound
// lookup waves, with no launch of their own.
//
// A convf1 work-group: a 4x16 pixel tile x 32 output channels; wave w owns
// channels 8w .. 8w+7 of the group for all 64 pixels (lane = pixel).  The
// group's weights (49 taps x 2 x 32, 12.5 KB, one coalesced copy) and the flow
// patch (10x22 pixels, zeros off the image) are staged in the LDS the lookup
// blocks use for their patches; per tap the lane reads its flow pair and the
// wave's 16 weights (broadcast reads) and accumulates 16 fp32 FMAs (packed).
// (Weights as wave-uniform scalar loads instead: each dy row waited on the
// scalar cache, 16.2 us per fused launch in the forward under rocprof.)  Exact
// fp32 products (the reference's fp32 conv, any summation order); the f16 /
// bf16 modes round the flow here and the weights on the host, as the MFMA
// kernels' operands.
// ============================================================================

__device__ __forceinline__ void flowconv_block(const FlowConvArgs& f, const LookupArgs& a, int bid, float* lds) {
  constexpr int KK = FC_MAXK * FC_MAXK;
  const int lane = threadIdx.x & 63;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  int t = bid;
  const int g = t % f.ngrp;
  t /= f.ngrp;
  const int tc = t % f.tx;
  t /= f.tx;
  const int tr = t % f.ty;
  const int b = t / f.ty;
  const int H = a.H, W = a.W, P = H * W;
  constexpr int pad = FC_MAXK / 2;
  const int y0 = tr * FC_TH - pad, x0 = tc * FC_TW - pad;
  // LDS: the group's weights [tap][ci][32] (12.5 KB), then the flow patch (10 x 22 float2)
  float* wl = lds;
  float2* fl = reinterpret_cast<float2*>(lds + KK * 2 * FC_CG);
  const f32x4* wsrc = reinterpret_cast<const f32x4*>(f.w + (long)g * KK * 2 * FC_CG);
  for (int i = threadIdx.x; i < KK * 2 * FC_CG / 4; i += 256) reinterpret_cast<f32x4*>(wl)[i] = wsrc[i];
  for (int i = threadIdx.x; i < FC_PH * FC_PW; i += 256) {
    const int yy = y0 + i / FC_PW, xx = x0 + i % FC_PW;
    float2 v = {0.f, 0.f};
    if ((unsigned)yy < (unsigned)H && (unsigned)xx < (unsigned)W) {
      float cx, cy;
      load_coords(a.coords, a.coords_layout, b, yy * W + xx, P, cx, cy);
      // the lookup's flow output: coords1 - coords0, the same two subtractions
      v.x = round_operand(cx - (float)xx, f.rnd);
      v.y = round_operand(cy - (float)yy, f.rnd);
    }
    fl[i] = v;
  }
  __syncthreads();
  const int ly = lane >> 4, lx = lane & 15;
  // this wave: channels 8*wv .. 8*wv+7 of the group, weights as wave-uniform (broadcast) LDS reads
  const float* ww = wl + wv * 8;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
#pragma unroll 1
  for (int dy = 0; dy < FC_MAXK; ++dy) {
    const float2* row = fl + (ly + dy) * FC_PW + lx;
    const float* wr = ww + dy * FC_MAXK * 2 * FC_CG;
#pragma unroll
    for (int dx = 0; dx < FC_MAXK; ++dx) {
      const float2 v = row[dx];
      const f32x4 w0a = *reinterpret_cast<const f32x4*>(wr + dx * 2 * FC_CG);
      const f32x4 w0b = *reinterpret_cast<const f32x4*>(wr + dx * 2 * FC_CG + 4);
      const f32x4 w1a = *reinterpret_cast<const f32x4*>(wr + dx * 2 * FC_CG + FC_CG);
      const f32x4 w1b = *reinterpret_cast<const f32x4*>(wr + dx * 2 * FC_CG + FC_CG + 4);
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] = fmaf(v.x, w0a[j], acc[j]);
        acc[4 + j] = fmaf(v.x, w0b[j], acc[4 + j]);
      }
#pragma unroll
      for (int j = 0; j < 4; ++j) {
        acc[j] = fmaf(v.y, w1a[j], acc[j]);
        acc[4 + j] = fmaf(v.y, w1b[j], acc[4 + j]);
      }
    }
  }
  const int oy = tr * FC_TH + ly, ox = tc * FC_TW + lx;
  if (oy >= H || ox >= W) return;
  const int c0 = g * FC_CG + wv * 8;
  float o[8];
  bool big = false;
#pragma unroll
  for (int j = 0; j < 8; ++j) {
    o[j] = fmaxf(acc[j] + (f.bias ? f.bias[c0 + j] : 0.f), 0.f);
    big |= o[j] > RAFT_RANGE_LIMIT;
  }
  if (f.range_flag && big) *f.range_flag = 1;
  float* dst = f.out + ((long)b * P + oy * W + ox) * f.out_ld + c0;
  *reinterpret_cast<f32x4*>(dst) = f32x4{o[0], o[1], o[2], o[3]};
  *reinterpret_cast<f32x4*>(dst + 4) = f32x4{o[4], o[5], o[6], o[7]};
}

// blocks [0, f.nblocks) of the F1 instantiation: convf1 tiles (above); the rest, and every
// block of the plain lookup: four query pixels, one per wave (pixel (blockIdx - nblocks)*4 + wave)
// SCAL: the window tests as scalar intervals (fewer VALU, more SALU per wave) for grids of
// at most two resident rounds, where a wave's latency sets the time; larger grids run the
// VALU form, since at 8 waves per SIMD the scalar unit becomes the limit (see below).
template <int R, int LMAX, bool F1, bool SCAL = false>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(8))) void corr_lookup_kernel(LookupArgs a,
                                                                                                 FlowConvArgs f) {
  __shared__ __attribute__((aligned(16))) float patch[4][16 * patch_rs<LMAX>()];
  __shared__ __attribute__((aligned(16))) int4 ytab[4][LMAX * (2 * R + 1)];  // y-entries: (w, t, 1 - t, floor)
  int bid = (int)blockIdx.x;
  if constexpr (F1) {
    static_assert(4 * 16 * patch_rs<LMAX>() >= FC_MAXK * FC_MAXK * 2 * FC_CG + 2 * FC_PW * FC_PH,
                  "convf1's weights and flow patch fit the lookup patches");
    if (bid < f.nblocks) {
      flowconv_block(f, a, bid, &patch[0][0]);
      return;
    }
    bid -= f.nblocks;
  }
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int RD = 2 * R + 1;
  constexpr int WD = 2 * R + 2;  // integer window (<= 10 -> <= 4 tiles per axis)
  constexpr int RS = patch_rs<LMAX>();  // patch row stride (floats)
  static_assert(WD <= 13, "window must fit 4 tiles");
  static_assert(LMAX * RD <= 64, "one lane per (level, x offset)");
  static_assert(RS + 16 <= 255, "ds_read2 offsets");
  const int lane = threadIdx.x & 63;
  const int P = a.H * a.W;
  // global pixel index b*P + p: wave-uniform, so the index math stays scalar (B*P < 2^30, host-checked)
  const int gp = bid * 4 + wv;
  const bool valid = gp < a.B * P;
  const int gpc = valid ? gp : 0;
  // (b, p) by a division only where a layout needs them: the forward's NHWC coords and
  // outputs index by gpc alone, and a division is ~30 instructions on the scalar unit,
  // which at B=8 is a co-limit of this kernel
  auto bp = [&](int& b, int& p) {
    b = gpc / P;
    p = gpc - b * P;
  };
  float x = 0.f, y = 0.f;
#ifdef LK_STAMPS
  const unsigned long long lk_r0 = lk_clock(true);
#endif
  LK_STAMP(0);
  if (a.coords_layout == 0) {
    x = a.coords[2L * gpc];
    y = a.coords[2L * gpc + 1];
  } else {
    int b, p;
    bp(b, p);
    load_coords(a.coords, a.coords_layout, b, p, P, x, y);
  }
#ifdef LK_STAMPS
  asm volatile("" ::"v"(x), "v"(y));
#endif
  LK_STAMP(1);

  // phase 1: per level, the <= 4x4 tiles covering the (2r+2)^2 integer window,
  // one 16-B load per lane (lane = tile row ti, tile col tj, row-in-tile rr),
  // all levels in flight together.  The window geometry is wave-uniform
  // (scalar); the pixel's map base too.
  const int ti = lane >> 4, tj = (lane >> 2) & 3, rr = lane & 3;
  const int lrow = ti * 4 + rr;  // the lane's row of the 16-row patch
  // phase 2's lane -> (level, offset) map and its level constants, loaded ahead of the tiles
  // (so waiting for them leaves the tile loads in flight)
  const int nlane = a.L * RD;
  const bool col = lane < nlane;
  // lane / RD by compares (3 VALU)
  int lq = 0;
#pragma unroll
  for (int k = 1; k < LMAX; ++k) lq += lane >= k * RD ? 1 : 0;
  const int l = col ? lq : 0;
  const int ix = lane - l * RD;
  const f32x4 prm = a.prm[l];
  f32x4 v[LMAX];
  // The window geometry is wave-uniform and comes from ONE float floor per axis:
  // floor(x / 2^k) = floor(floor(x) / 2^k) = floor(x) >> k, and x * 2^-k is exact, so every
  // level's window origin is an integer shift of level 0's (the same tiles as flooring
  // x * 2^-k per level; coords beyond the int range put both windows far off every map).
  // The per-level shifts then run on the SALU instead of four float floors + converts per
  // axis on the VALU.  (The builtin, not an inline-asm v_readfirstlane: issued right behind
  // the v_cvt that wrote its operand, the asm version read a stale value on gfx950 -- the
  // hazard recognizer does not look into asm -- and fetched wrong tiles.)
  const int xf = __builtin_amdgcn_readfirstlane((int)floorf(x));
  const int yf = __builtin_amdgcn_readfirstlane((int)floorf(y));
#pragma unroll
  for (int k = 0; k < LMAX; ++k) {
    const int x0 = (xf >> k) - R;
    const int y0 = (yf >> k) - R;
    const int tyo = y0 >> 2, txo = x0 >> 2;  // arithmetic shift = floor division by 4 (negative too)
    const int ntx = ((x0 + WD - 1) >> 2) - txo + 1;  // tile columns the window needs (3 or 4)
    const Level& lv = a.lv[k];
    __amdgpu_buffer_rsrc_t rs;
    unsigned off;
    if constexpr (SCAL) {
      // Fetched: the rows of the window's WD rows that lie on the map's tile rows, the
      // window's tile columns that lie on the map -- two scalar intervals, so a lane's test is
      // one subtract + one unsigned compare per axis: patch row lrow <-> map row tyo*4 + lrow
      // in [max(y0, 0), min(y0 + WD, 4 th)); tile column tj <-> txo + tj in
      // [max(txo, 0), min(txo + ntx, tw)).  (The interval origins through readfirstlane: one
      // SGPR each, so the test is not re-associated into two VALU adds.)
      const int rlo = max(y0, 0), rhi = min(y0 + WD, 4 * lv.th);
      const int clo = max(txo, 0), chi = min(txo + ntx, lv.tw);
      const int rb = __builtin_amdgcn_readfirstlane(rlo - 4 * tyo), cb = __builtin_amdgcn_readfirstlane(clo - txo);
      const bool ok = (k < a.L) & valid & ((unsigned)(lrow - rb) < (unsigned)max(rhi - rlo, 0)) &
                      ((unsigned)(tj - cb) < (unsigned)max(chi - clo, 0));
      // a raw buffer whose base is the window's first tile (tile (tyo, txo) of this pixel's
      // level map; before the map's start when the window hangs over its top or left edge): a
      // lane's byte offset is (ti tw + tj) 64 + 16 rr = ti (64 tw) + 16 (lane & 15); lanes
      // without a tile row to fetch pass an offset above num_records (zeros, no access; the
      // fetched lanes' offsets lie in the map by the tests above)
      const float* wb = a.lbase[k] + (long)((unsigned long long)(unsigned)gpc * (unsigned)lv.mapsz) +
                        ((long)tyo * lv.tw + txo) * 16;
      rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(wb), (short)0, 0x7FFFFFFF, 0x00020000);
      off = ok ? __umul24((unsigned)ti, (unsigned)(64 * lv.tw)) + 16u * (unsigned)(lane & 15) : 0x80000000u;
    } else {
      const int ty = tyo + ti, tx = txo + tj;
      // only tile rows inside the window's WD rows are fetched (that also bounds the tile
      // row count), only the window's tile columns, only tiles on the map.  (These tests stay
      // on the VALU: at 8 waves per SIMD the scalar unit is the other limit -- moving them to
      // scalar interval bounds cut VALU 290 -> 271 per wave but raised SALU 328 -> 406, and B=8
      // ran 8 % slower.)
      const bool ok = (k < a.L) & valid & (tj < ntx) & ((unsigned)(lrow + (tyo * 4 - y0)) < (unsigned)WD) &
                      ((unsigned)ty < (unsigned)lv.th) & ((unsigned)tx < (unsigned)lv.tw);
      // a raw buffer over this pixel's level map: lanes without a tile row to fetch pass an
      // out-of-range offset and get zeros (the map's zero padding) without a memory access.
      // (The map offset as one 32 x 32 -> 64-bit scalar product: mapsz < 2^31.)
      const float* mapb = a.lbase[k] + (long)((unsigned long long)(unsigned)gpc * (unsigned)lv.mapsz);
      rs = __builtin_amdgcn_make_buffer_rsrc(const_cast<float*>(mapb), (short)0, (int)(lv.mapsz * 4), 0x00020000);
      off = ok ? ((__umul24((unsigned)ty, (unsigned)lv.tw) + (unsigned)tx) * 64u + (unsigned)(rr * 16)) : 0x80000000u;
    }
#ifdef LK_ABL_NOLOAD  // timing ablation (dev builds only): no tile loads
    v[k] = f32x4{(float)off, 0.f, 0.f, 0.f};
#else
    v[k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
#endif
  }

  LK_STAMP(2);
  // phase 2 (while the loads fly): lane (l, d) = (lane / RD, lane % RD)
  // evaluates x-entry d (kept: this lane's column in phase 3) and y-entry d
  // (shared through LDS) of level l, with the reference's arithmetic — offset
  // added to the centroid, bilinear_sampler's 2x/(W-1)-1, grid_sample's
  // (g+1)*((W-1)/2) — so corner indices and weights are the reference's
  int xw, xi, yw;
  float xt;
  {
    const float wm1 = prm[0], rw = prm[1], hm1 = prm[2], rh = prm[3];
    const float s = __builtin_ldexpf(1.0f, -l);
    axis_entry<R>(x * s, xf >> l, ix, wm1, rw, xw, xt, xi);
    int yi;
    float yt;
    axis_entry<R>(y * s, yf >> l, ix, hm1, rh, yw, yt, yi);
    // .x: the row's byte offset in the patch (row * RS * 4), or the negative OFF_PATCH / NAN_POS code
    if (col) ytab[wv][lane] = int4{yw >= 0 ? yw * RS * 4 : yw, __float_as_int(yt), __float_as_int(1.0f - yt), yi};
  }
  // (lanes that fetched nothing hold zeros from the out-of-range buffer load)
#pragma unroll
  for (int k = 0; k < LMAX; ++k) *reinterpret_cast<f32x4*>(&patch[wv][pidx<LMAX>(lrow, tj * 4, k)]) = v[k];
  LK_STAMP(3);
  // the patch and y-table are this wave's own: a wave-local barrier (the
  // block's four pixels never wait for each other)
  __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
  __builtin_amdgcn_wave_barrier();
  __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
  if (!valid) return;

  // phase 3: lane (l, ix) walks its column iy = 0 .. 2r of output channels
  // l*RD^2 + ix*RD + iy; the y-entries are LDS broadcasts.  Bilinear as two horizontal
  // interpolations and a vertical one, with fused multiply-adds (within 2 ulp of the
  // reference's four products: the parity bound of the lookup is 1e-5 on O(1..10) values)
  const int ntap = a.L * RD * RD;
  const int cbase = l * RD * RD + ix * RD;
  const float ex = 1.0f - xt;
  float val[RD];
  // the common case: every entry of the wave is finite and on the patch
  if (__all(!col || (xw >= 0 && yw >= 0))) {
    if (col) {
      const char* p0 = reinterpret_cast<const char*>(&patch[wv][pidx<LMAX>(0, xw, l)]);
      const char* p1 = reinterpret_cast<const char*>(&patch[wv][pidx<LMAX>(0, xw + 1, l)]);
      auto at = [](const char* b, int byte) { return *reinterpret_cast<const float*>(b + byte); };
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) {
        const int4 ye = ytab[wv][l * RD + iy];
        const int ro = ye.x;
        const float ty = __int_as_float(ye.y), sS = __int_as_float(ye.z);
        // (h0, h1) = the two rows' horizontal interpolations as one packed pair: each
        // ds_read2 returns a column's two rows in consecutive registers, so the pair
        // needs no repacking (v_pk_mul + v_pk_fma, the same roundings as two fmaf)
        const f32x2 c0 = {at(p0, ro), at(p0, ro + 4 * RS)}, c1 = {at(p1, ro), at(p1, ro + 4 * RS)};
        const f32x2 hh = __builtin_elementwise_fma(c0, (f32x2){ex, ex}, c1 * (f32x2){xt, xt});
        val[iy] = fmaf(sS, hh.x, ty * hh.y);
      }
    }
  } else if (col) {
    unsigned deferred = 0;
#pragma unroll
    for (int iy = 0; iy < RD; ++iy) {
      const int4 ye = ytab[wv][l * RD + iy];
      const int yw2 = ye.x;  // row * RS * 4 (bytes), or a negative code
      const float ty = __int_as_float(ye.y), sS = __int_as_float(ye.z);
      const bool on = (xw | yw2) >= 0;
      const bool nan = xw == NAN_POS || yw2 == NAN_POS;
      const int r0 = on ? yw2 / (4 * RS) : 0, c0 = on ? xw : 0;
      const float* pl = &patch[wv][0];
      const float v = pl[pidx<LMAX>(r0, c0, l)] * (sS * ex) + pl[pidx<LMAX>(r0, c0 + 1, l)] * (sS * xt) +
                      pl[pidx<LMAX>(r0 + 1, c0, l)] * (ty * ex) + pl[pidx<LMAX>(r0 + 1, c0 + 1, l)] * (ty * xt);
      val[iy] = nan ? __builtin_nanf("") : v;
      deferred |= (!on && !nan) ? 1u << iy : 0u;
    }
    if (deferred != 0) {
      // taps whose floor the float round trip moved off the staged patch: the
      // four corners from global memory (zeros outside the map)
      const Level& lv = a.lv[l];
      const float* m = a.pyr + lv.off + (long)gp * lv.mapsz;
      auto at = [&](int yy, int xx) {
        return ((unsigned)yy < (unsigned)lv.h && (unsigned)xx < (unsigned)lv.w) ? m[tiled_index(yy, xx, lv.tw)] : 0.f;
      };
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) {
        if (!((deferred >> iy) & 1u)) continue;
        const int4 ye = ytab[wv][l * RD + iy];
        const int yi = ye.w;
        const float ty = __int_as_float(ye.y), sS = __int_as_float(ye.z);
        val[iy] = at(yi, xi) * (sS * ex) + at(yi, xi + 1) * (sS * xt) + at(yi + 1, xi) * (ty * ex) +
                  at(yi + 1, xi + 1) * (ty * xt);
      }
    }
  }
  LK_STAMP(4);
  if (a.range_flag && col) {  // f16x3 range guard: the output feeds the split-precision convc1
    float mx = fabsf(val[0]);
#pragma unroll
    for (int iy = 1; iy < RD; ++iy) mx = fmaxf(mx, fabsf(val[iy]));
    if (mx > RAFT_RANGE_LIMIT) *a.range_flag = 1;
  }
#ifdef LK_ABL_NOSTORE  // timing ablation (dev builds only): no output stores
  if (val[0] != -12345.f) return;
#endif
  const bool vec_out = a.out_layout == 0 && (a.out_ld & 3) == 0 && (ntap & 3) == 0 && ((uintptr_t)a.out & 15) == 0;
  if (vec_out) {
    // NHWC row: transpose the columns through this wave's (consumed) patch
    // and write the row with 16-B stores (a one-dword-per-lane strided store
    // tail costs more than the gather itself)
    float* st = &patch[wv][0];
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    if (col) {
#pragma unroll
      for (int iy = 0; iy < RD; ++iy) st[cbase + iy] = val[iy];
    }
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float* orow = a.out + (long)gp * a.out_ld;
    for (int j = 4 * lane; j < ntap; j += 256)
      *reinterpret_cast<f32x4*>(orow + j) = *reinterpret_cast<const f32x4*>(st + j);
  } else if (col) {
    int b, p;
    bp(b, p);
    float* orow = a.out_layout == 0 ? a.out + (long)gp * a.out_ld + cbase
                                    : a.out + ((long)b * ntap + cbase) * P + p;
    const long ostep = a.out_layout == 0 ? 1 : P;
#pragma unroll
    for (int iy = 0; iy < RD; ++iy) orow[iy * ostep] = val[iy];
  }
  if (a.flow && lane < 2) {
    int b, p;
    bp(b, p);
    const float g = lane == 0 ? (float)(p % a.W) : (float)(p / a.W);
    a.flow[(long)gp * a.flow_ld + lane] = (lane == 0 ? x : y) - g;
  }
#ifdef LK_STAMPS
  LK_STAMP(5);
  const unsigned long long lk_r1 = lk_clock(true);
  if (lane == 0 && gp < 65536) {
    unsigned long long* g = g_lkstamp + gp * 8;
    g[0] = lk_r0;
    g[1] = lk_r1;
    g[2] = lk_t1 - lk_t0;  // coords load
    g[3] = lk_t2 - lk_t1;  // tile-load issue
    g[4] = lk_t3 - lk_t2;  // phase 2 + landing of the tiles + patch writes
    g[5] = lk_t4 - lk_t3;  // taps
    g[6] = lk_t5 - lk_t4;  // stores (issued and completed)
  }
#endif
}



// Any radius / level count (the reference's CorrBlock takes any r; RAFT's r = 3, 4 use the
// kernel above): one thread per (query pixel, level, output channel), the same per-axis
// arithmetic as axis_entry, corners read from the tiled maps (zeros off the map; NaN where
// the position is not finite, as the reference on a 1-px level).
__global__ void corr_lookup_generic_kernel(LookupArgs a) {
#pragma clang fp contract(off)
  const int r = a.r, rd = 2 * r + 1, ntap = a.L * rd * rd;
  const int P = a.H * a.W;
  const long total = (long)a.B * P * ntap;
  for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
    const int ch = (int)(i % ntap);
    const long gp = i / ntap;
    const int b = (int)(gp / P), p = (int)(gp - (long)b * P);
    const int l = ch / (rd * rd), k = ch - l * rd * rd;
    const int ix = k / rd, iy = k - ix * rd;  // channel lvl*rd^2 + ix*rd + iy, ix moves x
    float x, y;
    load_coords(a.coords, a.coords_layout, b, p, P, x, y);
    const float s = 1.0f / (float)(1 << l);
    const float m1x = a.wm1[l], m1y = a.hm1[l];
    const float X = x * s + (float)(ix - r), Y = y * s + (float)(iy - r);
    const float ux = (div_rn(2.0f * X, m1x, a.rw[l]) - 1.0f + 1.0f) * (m1x * 0.5f);
    const float uy = (div_rn(2.0f * Y, m1y, a.rh[l]) - 1.0f + 1.0f) * (m1y * 0.5f);
    float v;
    if (!isfinite(ux) || !isfinite(uy)) {
      v = __builtin_nanf("");
    } else {
      const float fx = floorf(ux), fy = floorf(uy);
      const float tx = ux - fx, ty = uy - fy;
      const int x0 = (int)fx, y0 = (int)fy;
      const Level& lv = a.lv[l];
      const float* m = a.pyr + lv.off + gp * lv.mapsz;
      auto at = [&](int yy, int xx) {
        return ((unsigned)yy < (unsigned)lv.h && (unsigned)xx < (unsigned)lv.w) ? m[tiled_index(yy, xx, lv.tw)] : 0.f;
      };
      const float ex = 1.0f - tx, sS = 1.0f - ty;
      v = at(y0, x0) * (sS * ex) + at(y0, x0 + 1) * (sS * tx) + at(y0 + 1, x0) * (ty * ex) +
          at(y0 + 1, x0 + 1) * (ty * tx);
    }
    if (a.range_flag && fabsf(v) > RAFT_RANGE_LIMIT) *a.range_flag = 1;
    if (a.out_layout == 0)
      a.out[gp * a.out_ld + ch] = v;
    else
      a.out[((long)b * ntap + ch) * P + p] = v;
    if (a.flow && ch < 2) a.flow[gp * a.flow_ld + ch] = (ch == 0 ? x : y) - (ch == 0 ? (float)(p % a.W) : (float)(p / a.W));
  }
}

int grid_for(long n, int block = 256) {
  long g = (n + block - 1) / block;
  if (g > 65536) g = 65536;
  if (g < 1) g = 1;
  return (int)g;
}

// level geometry; returns false if a level is empty
bool pyramid_levels(int B, int H, int W, int L, Level* lv) {
  long off = 0;
  int h = H, w = W;
  const long P = (long)H * W;
  for (int l = 0; l < L; ++l) {
    if (h < 1 || w < 1) return false;
    lv[l].h = h;
    lv[l].w = w;
    lv[l].th = cdiv(h, 4);
    lv[l].tw = cdiv(w, 4);
    lv[l].mapsz = (long)lv[l].th * lv[l].tw * 16;
    lv[l].off = off;
    off += (long)B * P * lv[l].mapsz;
    h /= 2;
    w /= 2;
  }
  return true;
}

}  // namespace
}  // namespace raft

using namespace raft;

#ifdef LK_STAMPS
extern "C" int raft_debug_lkstamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lkstamp), sizeof(unsigned long long) * (size_t)n);
}
#endif

extern "C" size_t raft_corr_pyramid_floats(int B, int H, int W, int L) {
  if (B <= 0 || H <= 0 || W <= 0 || L <= 0 || L > LK_MAXL) return 0;
  Level lv[LK_MAXL];
  if (!pyramid_levels(B, H, W, L, lv)) return 0;
  return (size_t)(lv[L - 1].off + (long)B * H * W * lv[L - 1].mapsz);
}

extern "C" int raft_corr_build(const float* fmap1, const float* fmap2, int ld, int B, int H, int W, int C, int L,
                               float sqrt_c, float* pyramid, raft_stream_t stream) {
  return raft_corr_build_prec(fmap1, fmap2, ld, B, H, W, C, L, sqrt_c, RAFT_PREC_FP32, pyramid, stream);
}

extern "C" int raft_corr_build_prec(const float* fmap1, const float* fmap2, int ld, int B, int H, int W, int C, int L,
                                    float sqrt_c, int precision, float* pyramid, raft_stream_t stream) {
  using namespace raft;
  RAFT_REQUIRE(precision == RAFT_PREC_FP32 || precision == RAFT_PREC_F16X3,
               "raft_corr_build_prec: precision must be RAFT_PREC_FP32 or RAFT_PREC_F16X3 (got %d)", precision);
  RAFT_REQUIRE(fmap1 && fmap2 && pyramid, "raft_corr_build: null pointer");
  RAFT_REQUIRE(B > 0 && H > 0 && W > 0 && C > 0 && L >= 1 && L <= LK_MAXL, "raft_corr_build: bad sizes");
  RAFT_REQUIRE(C % 4 == 0, "raft_corr_build: C must be a multiple of 4 (got %d)", C);
  RAFT_REQUIRE(ld % 4 == 0 && ld >= C, "raft_corr_build: ld must be >= C and a multiple of 4");
  RAFT_REQUIRE((((uintptr_t)fmap1 | (uintptr_t)fmap2 | (uintptr_t)pyramid) & 15) == 0,
               "raft_corr_build: fmaps and pyramid must be 16-byte aligned");
  Level lv[LK_MAXL];
  RAFT_REQUIRE(pyramid_levels(B, H, W, L, lv), "raft_corr_build: a pyramid level is empty (%dx%d, %d levels)", H, W, L);
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
  a.pyr = pyramid;
  a.l0 = lv[0];
  a.has_l1 = L > 1;
  a.l1 = lv[L > 1 ? 1 : 0];
  a.nbx = cdiv(W, 8);
  {
    // non-temporal pyramid stores when level 0 alone is far past the 256 MiB Infinity Cache (the
    // lookups then read it from HBM either way); RAFT_CORR_NT=0 / 1 overrides
    const char* e = getenv("RAFT_CORR_NT");
    const double l0_bytes = 4.0 * B * (double)P * lv[0].mapsz;
    a.nt = e && (e[0] == '0' || e[0] == '1') ? e[0] == '1' : l0_bytes > 512.0 * 1024 * 1024;
  }
  hipStream_t s = as_stream(stream);
  static const bool big = [] {
    const char* e = getenv("RAFT_CORR_BUILD_BIG");
    return !(e && e[0] == '0');
  }();
  if (precision == RAFT_PREC_FP32) {
    dim3 grid(cdiv((int)P, CB_BM), cdiv(H, 8) * a.nbx, B);
    hipLaunchKernelGGL(corr_build_kernel<false>, grid, dim3(256), 0, s, a);
  } else if (big) {  // 16-B epilogue stores (the pyramid is 16-B aligned, checked above)
    a.B = B;
    a.mt = cdiv((int)P, CB2_BM);
    a.ntl = cdiv(H, 8) * cdiv(W, 16);
    a.gm = a.mt;  // M tiles fastest over the whole batch image
    a.nfast = 0;
    a.xcd = 0;
    if (const char* e = getenv("RAFT_CB_ORDER")) {  // "gm,nfast,xcd" (tile-order experiments)
      int gm = 0, nf = 0, xc = 0;
      if (sscanf(e, "%d,%d,%d", &gm, &nf, &xc) == 3 && gm > 0) {
        a.gm = min(gm, a.mt);
        a.nfast = nf != 0;
        a.xcd = xc != 0;
      }
    }
    const dim3 grid((unsigned)((long)B * a.mt * a.ntl));
    hipLaunchKernelGGL(corr_build2_kernel, grid, dim3(512), 0, s, a);
  } else {
    dim3 grid(cdiv((int)P, CB_BM), cdiv(H, 8) * a.nbx, B);
    hipLaunchKernelGGL(corr_build_kernel<true>, grid, dim3(256), 0, s, a);
  }
  int rc = check_launch("raft_corr_build");
  if (rc) return rc;
  for (int l = 2; l < L; ++l) {
    const long n = (long)B * P * lv[l].mapsz;
    hipLaunchKernelGGL(pool2_tiled_kernel, dim3(grid_for(n)), dim3(256), 0, s, pyramid, pyramid, (long)B * P, lv[l - 1],
                       lv[l]);
    rc = check_launch("raft_corr_build(pool)");
    if (rc) return rc;
  }
  return 0;
}

#ifdef CB4_STAMPS
extern "C" int raft_debug_cb4stamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_cb4stamp), sizeof(unsigned long long) * (size_t)n);
}
#endif

extern "C" size_t raft_corr_build_ws_bytes(int B, int H, int W, int C) {
  if (B <= 0 || H <= 0 || W <= 0 || C <= 0) return 0;
  return 2 * (size_t)B * H * W * C * 4 + 4096;  // the two split maps + the epilogue sink
}

namespace raft {
// whether raft_corr_build_ws takes the 256 x 256 kernel (corr_build4) for this shape: f16x3, C a multiple of
// 16 with >= 4 half-steps, 32-bit map offsets, RAFT_CORR_BUILD4 not 0 (the operand checks -- ld, alignment,
// a workspace -- come on top, per call)
static bool corr_build4_shape(int B, int H, int W, int C, int precision) {
  const char* e = getenv("RAFT_CORR_BUILD4");
  if (e && e[0] == '0') return false;
  return precision == RAFT_PREC_F16X3 && C % 16 == 0 && C >= 64 && C <= 1024 && B > 0 && H > 0 && W > 0 &&
         (double)B * H * W * C * 4 < 2147483648.0;
}
}  // namespace raft

extern "C" size_t raft_corr_build_ws_bytes_prec(int B, int H, int W, int C, int precision) {
  return raft::corr_build4_shape(B, H, W, C, precision) ? raft_corr_build_ws_bytes(B, H, W, C) : 0;
}

extern "C" int raft_corr_build_ws(const float* fmap1, const float* fmap2, int ld, int B, int H, int W, int C, int L,
                                  float sqrt_c, int precision, float* pyramid, void* ws, size_t ws_bytes,
                                  raft_stream_t stream) {
  using namespace raft;
  const long P = (long)H * W;
  // the 256 x 256 kernel where corr_build4_shape says so (raft_corr_build_ws_bytes_prec: its workspace) and
  // the operands fit it (no workspace, or an operand off 16-B alignment: the other kernel, as in ABI 14)
  const bool fits = corr_build4_shape(B, H, W, C, precision) && ld % 4 == 0 && ld >= C && ws != nullptr &&
                    (((uintptr_t)fmap1 | (uintptr_t)fmap2 | (uintptr_t)pyramid | (uintptr_t)ws) & 15) == 0;
  if (!fits) return raft_corr_build_prec(fmap1, fmap2, ld, B, H, W, C, L, sqrt_c, precision, pyramid, stream);
  RAFT_REQUIRE(fmap1 && fmap2 && pyramid, "raft_corr_build_ws: null pointer");
  RAFT_REQUIRE(B > 0 && H > 0 && W > 0 && L >= 1 && L <= LK_MAXL, "raft_corr_build_ws: bad sizes");
  RAFT_REQUIRE(ws_bytes >= raft_corr_build_ws_bytes(B, H, W, C), "raft_corr_build_ws: workspace too small "
               "(raft_corr_build_ws_bytes)");
  RAFT_REQUIRE((((uintptr_t)fmap1 | (uintptr_t)fmap2 | (uintptr_t)pyramid | (uintptr_t)ws) & 15) == 0,
               "raft_corr_build_ws: fmaps, pyramid and workspace must be 16-byte aligned");
  Level lv[LK_MAXL];
  RAFT_REQUIRE(pyramid_levels(B, H, W, L, lv), "raft_corr_build_ws: a pyramid level is empty (%dx%d, %d levels)", H,
               W, L);
  hipStream_t s = as_stream(stream);
  const size_t map_bytes = (size_t)B * P * C * 4;
  char* s1 = static_cast<char*>(ws);
  char* s2 = s1 + map_bytes;
  const long nq = (long)B * P * (C / 4);
  hipLaunchKernelGGL(corr_split4_kernel, dim3((unsigned)cdiv_l(nq, 256)), dim3(256), 0, s, fmap1, ld, (long)B * P, C, s1);
  hipLaunchKernelGGL(corr_split4_kernel, dim3((unsigned)cdiv_l(nq, 256)), dim3(256), 0, s, fmap2, ld, (long)B * P, C, s2);
  int rc = check_launch("raft_corr_build_ws(split)");
  if (rc) return rc;
  CB4Args a;
  a.s1 = s1;
  a.s2 = s2;
  a.sbytes = (unsigned)map_bytes;
  a.H = H;
  a.W = W;
  a.P = (int)P;
  a.nh = C / 16;
  a.sqrt_c = sqrt_c;
  a.pyr = pyramid;
  a.l0 = lv[0];
  a.l1 = lv[L > 1 ? 1 : 0];
  a.l2 = lv[L > 2 ? 2 : 0];
  // level 2 from the build's registers (RAFT_CB4_L2=0: from level 1 by pool2_tiled_kernel, the same bytes)
  static const bool l2_on = [] {
    const char* e = getenv("RAFT_CB4_L2");
    return !(e && e[0] == '0');
  }();
  const bool l2 = l2_on && L > 2;
  {
    const char* e = getenv("RAFT_CORR_NT");
    const double l0_bytes = 4.0 * B * (double)P * lv[0].mapsz;
    a.nt = e && (e[0] == '0' || e[0] == '1') ? e[0] == '1' : l0_bytes > 512.0 * 1024 * 1024;
  }
  // RAFT_CB4_W4=1: 4-wave work-groups, two per CU (r05p: config 2's map 156 -> 142 us alone, config 4's
  // 1.50 -> 1.54 ms, config 5's 2.47 -> 2.80 ms: the half-size units move 1.5x the operand bytes per
  // flop; the forward unchanged at config 2, 1.5 % slower at config 5), default: 8 waves, one per CU
  // (read per call, like RAFT_CB_ORDER: a test can switch it; a plan captures the launch it made)
  const bool w4 = [] {
    const char* e = getenv("RAFT_CB4_W4");
    return e && e[0] == '1';
  }();
  a.qt = (int)cdiv_l(P, w4 ? CB4_T / 2 : CB4_T);
  a.ttx = cdiv(W, 16);
  a.tt = cdiv(H, 16) * a.ttx;
  a.units = (long)B * a.qt * a.tt;
  a.sink = reinterpret_cast<f32x4*>(s2 + map_bytes);
  int cus = 256, dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess ||
      cus <= 0)
    cus = 256;
  // persistent: one 8-wave work-group per CU (128 KiB LDS) or two 4-wave ones (72 KiB each)
  const long wgs = w4 ? 2L * cus : (long)cus;
  const dim3 grid((unsigned)(a.units < wgs ? a.units : wgs));
  if (w4) {
    if (l2)
      hipLaunchKernelGGL((corr_build4_kernel<true, true, 4>), grid, dim3(256), 0, s, a);
    else if (L > 1)
      hipLaunchKernelGGL((corr_build4_kernel<true, false, 4>), grid, dim3(256), 0, s, a);
    else
      hipLaunchKernelGGL((corr_build4_kernel<false, false, 4>), grid, dim3(256), 0, s, a);
  } else if (l2) {
    hipLaunchKernelGGL((corr_build4_kernel<true, true>), grid, dim3(512), 0, s, a);
  } else if (L > 1) {
    hipLaunchKernelGGL(corr_build4_kernel<true>, grid, dim3(512), 0, s, a);
  } else {
    hipLaunchKernelGGL(corr_build4_kernel<false>, grid, dim3(512), 0, s, a);
  }
  rc = check_launch("raft_corr_build_ws");
  if (rc) return rc;
  for (int l = l2 ? 3 : 2; l < L; ++l) {
    const long n = (long)B * P * lv[l].mapsz;
    hipLaunchKernelGGL(pool2_tiled_kernel, dim3(grid_for(n)), dim3(256), 0, s, pyramid, pyramid, (long)B * P, lv[l - 1],
                       lv[l]);
    rc = check_launch("raft_corr_build_ws(pool)");
    if (rc) return rc;
  }
  return 0;
}

extern "C" int raft_corr_pyramid_level(const float* pyramid, int B, int H, int W, int L, int level, float* out,
                                       raft_stream_t stream) {
  RAFT_REQUIRE(pyramid && out && B > 0 && H > 0 && W > 0 && L >= 1 && L <= LK_MAXL && level >= 0 && level < L,
               "raft_corr_pyramid_level: bad arguments");
  Level lv[LK_MAXL];
  RAFT_REQUIRE(pyramid_levels(B, H, W, L, lv), "raft_corr_pyramid_level: a pyramid level is empty");
  const long n = (long)B * H * W * lv[level].h * lv[level].w;
  hipLaunchKernelGGL(untile_kernel, dim3(grid_for(n)), dim3(256), 0, as_stream(stream), pyramid, out,
                     (long)B * H * W, lv[level]);
  return check_launch("raft_corr_pyramid_level");
}

namespace raft {
// validated LookupArgs of a raft_corr_lookup call (0, or the error code)
int lookup_args(LookupArgs& a, const float* pyramid, int B, int H, int W, int L, int radius, const float* coords,
                int coords_layout, float* out, int out_ld, int out_layout, float* flow_out, int flow_ld,
                int* range_flag) {
  RAFT_REQUIRE(pyramid && coords && out, "raft_corr_lookup: null pointer");
  RAFT_REQUIRE(B > 0 && H > 0 && W > 0 && L >= 1 && L <= LK_MAXL, "raft_corr_lookup: bad sizes");
  RAFT_REQUIRE(radius >= 0 && radius <= 32, "raft_corr_lookup: radius must be 0..32 (got %d)", radius);
  RAFT_REQUIRE(coords_layout == 0 || coords_layout == 1, "raft_corr_lookup: bad coords_layout");
  RAFT_REQUIRE(out_layout == 0 || out_layout == 1, "raft_corr_lookup: bad out_layout");
  const int rd = 2 * radius + 1;
  RAFT_REQUIRE(out_layout == 1 || out_ld >= L * rd * rd, "raft_corr_lookup: out_ld < L*(2r+1)^2");
  RAFT_REQUIRE(!flow_out || flow_ld >= 2, "raft_corr_lookup: flow_ld < 2");
  RAFT_REQUIRE(((uintptr_t)pyramid & 15) == 0, "raft_corr_lookup: pyramid must be 16-byte aligned");
  RAFT_REQUIRE((long)B * H * W < (1L << 30), "raft_corr_lookup: more than 2^30 query pixels (split the batch)");
  RAFT_REQUIRE((long)H * W * 16 * 4 < (1L << 31), "raft_corr_lookup: a per-pixel map exceeds 2 GiB");
  RAFT_REQUIRE(pyramid_levels(B, H, W, L, a.lv), "raft_corr_lookup: a pyramid level is empty");
  for (int l = L; l < LK_MAXL; ++l) a.lv[l] = a.lv[L - 1];
  for (int l = 0; l < LK_MAXL; ++l) {
    a.wm1[l] = (float)(a.lv[l].w - 1);
    a.hm1[l] = (float)(a.lv[l].h - 1);
    volatile float one = 1.0f;  // host IEEE division, as the reference's 1 / (W - 1) path on the device
    a.rw[l] = one / a.wm1[l];
    a.rh[l] = one / a.hm1[l];
    a.prm[l] = f32x4{a.wm1[l], a.rw[l], a.hm1[l], a.rh[l]};
  }
  a.pyr = pyramid;
  for (int l = 0; l < LK_MAXL; ++l) a.lbase[l] = pyramid + a.lv[l].off;
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
  a.range_flag = range_flag;
  return 0;
}

// The 4-level lookup: the scalar-interval form (SCAL) when the query pixels fill at most
// two resident rounds of lookup waves (latency-bound: B=1 9.8 -> 9.0 us at config 2), the
// VALU form beyond (scalar-unit-bound at full occupancy: B=8 44.7 vs 41-43 us).
template <int RR, bool F1>
void launch_lookup4(dim3 grid, hipStream_t s, const LookupArgs& a, const FlowConvArgs& f) {
  if (RR == 4 && (long)a.B * a.H * a.W <= 16384)
    hipLaunchKernelGGL((corr_lookup_kernel<RR, 4, F1, RR == 4>), grid, dim3(256), 0, s, a, f);
  else
    hipLaunchKernelGGL((corr_lookup_kernel<RR, 4, F1>), grid, dim3(256), 0, s, a, f);
}
}  // namespace raft

extern "C" int raft_corr_lookup(const float* pyramid, int B, int H, int W, int L, int radius, const float* coords,
                                int coords_layout, float* out, int out_ld, int out_layout, float* flow_out,
                                int flow_ld, int* range_flag, raft_stream_t stream) {
  LookupArgs a;
  const int rc = lookup_args(a, pyramid, B, H, W, L, radius, coords, coords_layout, out, out_ld, out_layout, flow_out,
                             flow_ld, range_flag);
  if (rc) return rc;
  const int rd = 2 * radius + 1;
  dim3 grid((unsigned)cdiv_l((long)B * H * W, 4));
  hipStream_t s = as_stream(stream);
  if (radius > 4 || radius < 1) {  // any other radius: the generic kernel
    hipLaunchKernelGGL(corr_lookup_generic_kernel, dim3(grid_for((long)B * H * W * L * rd * rd)), dim3(256), 0, s, a);
    return check_launch("raft_corr_lookup(generic radius)");
  }
  // the 4-level case (RAFT) gets a tight instantiation; other level counts use LMAX = 6
#define RAFT_LOOKUP_CASE(RR)                                                           \
  case RR:                                                                             \
    if (L <= 4)                                                                        \
      launch_lookup4<RR, false>(grid, s, a, FlowConvArgs{});                           \
    else                                                                               \
      hipLaunchKernelGGL((corr_lookup_kernel<RR, LK_MAXL, false>), grid, dim3(256), 0, s, a, FlowConvArgs{}); \
    break;
  switch (radius) {
    RAFT_LOOKUP_CASE(1)
    RAFT_LOOKUP_CASE(2)
    RAFT_LOOKUP_CASE(3)
    default:
    RAFT_LOOKUP_CASE(4)
  }
#undef RAFT_LOOKUP_CASE
  return check_launch("raft_corr_lookup");
}

namespace raft {
// validated FlowConvArgs of a convf1 call (0, or the error code); who = the entry point's name
int flowconv_args(FlowConvArgs& f, const char* who, int B, int H, int W, const float* f1_weight, const float* f1_bias,
                  int f1_n, int f1_k, int f1_precision, float* f1_out, int f1_out_ld, int* f1_range_flag) {
  RAFT_REQUIRE(f1_weight && f1_out, "%s: null convf1 pointer", who);
  RAFT_REQUIRE(f1_k == FC_MAXK, "%s: kernel size must be 7 (got %d)", who, f1_k);
  RAFT_REQUIRE(f1_n > 0 && f1_n % FC_CG == 0, "%s: output channels must be a multiple of 32 (got %d)", who, f1_n);
  RAFT_REQUIRE(f1_out_ld >= f1_n && f1_out_ld % 4 == 0 && (((uintptr_t)f1_out | (uintptr_t)f1_weight) & 15) == 0,
               "%s: weight and output rows must be 16-byte aligned (ld >= n, ld %% 4 == 0)", who);
  RAFT_REQUIRE(f1_precision == RAFT_PREC_FP32 || f1_precision == RAFT_PREC_F16X3 || f1_precision == RAFT_PREC_F16 ||
                   f1_precision == RAFT_PREC_BF16,
               "%s: bad precision %d", who, f1_precision);
  f.w = f1_weight;
  f.bias = f1_bias;
  f.out = f1_out;
  f.out_ld = f1_out_ld;
  f.n = f1_n;
  f.k = f1_k;
  f.rnd = f1_precision == RAFT_PREC_F16 ? 1 : f1_precision == RAFT_PREC_BF16 ? 2 : 0;
  f.range_flag = f1_range_flag;
  f.tx = cdiv(W, FC_TW);
  f.ty = cdiv(H, FC_TH);
  f.ngrp = f1_n / FC_CG;
  const long nb = (long)B * f.tx * f.ty * f.ngrp;
  RAFT_REQUIRE(nb + cdiv_l((long)B * H * W, 4) < (1L << 31), "%s: grid too large", who);
  f.nblocks = (int)nb;
  return 0;
}
}  // namespace raft

extern "C" int raft_corr_lookup_convf1(const float* pyramid, int B, int H, int W, int L, int radius,
                                       const float* coords, int coords_layout, float* out, int out_ld, int out_layout,
                                       float* flow_out, int flow_ld, int* range_flag, const float* f1_weight,
                                       const float* f1_bias, int f1_n, int f1_k, int f1_precision, float* f1_out,
                                       int f1_out_ld, int* f1_range_flag, raft_stream_t stream) {
  LookupArgs a;
  int rc = lookup_args(a, pyramid, B, H, W, L, radius, coords, coords_layout, out, out_ld, out_layout, flow_out,
                       flow_ld, range_flag);
  if (rc) return rc;
  FlowConvArgs f;
  rc = flowconv_args(f, "raft_corr_lookup_convf1", B, H, W, f1_weight, f1_bias, f1_n, f1_k, f1_precision, f1_out,
                     f1_out_ld, f1_range_flag);
  if (rc) return rc;
  hipStream_t s = as_stream(stream);
  const unsigned nlk = (unsigned)cdiv_l((long)B * H * W, 4);
  if (radius > 4 || radius < 1) {  // the generic lookup, then the convf1 blocks alone
    rc = raft_corr_lookup(pyramid, B, H, W, L, radius, coords, coords_layout, out, out_ld, out_layout, flow_out,
                          flow_ld, range_flag, stream);
    if (rc) return rc;
    hipLaunchKernelGGL((corr_lookup_kernel<4, 4, true>), dim3(f.nblocks), dim3(256), 0, s, a, f);
    return check_launch("raft_corr_lookup_convf1(convf1)");
  }
  const dim3 grid((unsigned)f.nblocks + nlk);
#define RAFT_LOOKUP_F1_CASE(RR)                                                                \
  case RR:                                                                                     \
    if (L <= 4)                                                                                \
      launch_lookup4<RR, true>(grid, s, a, f);                                                 \
    else                                                                                       \
      hipLaunchKernelGGL((corr_lookup_kernel<RR, LK_MAXL, true>), grid, dim3(256), 0, s, a, f); \
    break;
  switch (radius) {
    RAFT_LOOKUP_F1_CASE(1)
    RAFT_LOOKUP_F1_CASE(2)
    RAFT_LOOKUP_F1_CASE(3)
    default:
    RAFT_LOOKUP_F1_CASE(4)
  }
#undef RAFT_LOOKUP_F1_CASE
  return check_launch("raft_corr_lookup_convf1");
}

extern "C" int raft_convf1_flow(const float* coords, int coords_layout, int B, int H, int W, const float* f1_weight,
                                const float* f1_bias, int f1_n, int f1_k, int f1_precision, float* f1_out,
                                int f1_out_ld, int* f1_range_flag, raft_stream_t stream) {
  RAFT_REQUIRE(coords && B > 0 && H > 0 && W > 0, "raft_convf1_flow: bad arguments");
  RAFT_REQUIRE(coords_layout == 0 || coords_layout == 1, "raft_convf1_flow: bad coords_layout");
  RAFT_REQUIRE((long)B * H * W < (1L << 30), "raft_convf1_flow: more than 2^30 pixels");
  FlowConvArgs f;
  const int rc = flowconv_args(f, "raft_convf1_flow", B, H, W, f1_weight, f1_bias, f1_n, f1_k, f1_precision, f1_out,
                               f1_out_ld, f1_range_flag);
  if (rc) return rc;
  LookupArgs a{};  // the convf1 blocks read only the coords and the geometry
  a.coords = coords;
  a.coords_layout = coords_layout;
  a.B = B;
  a.H = H;
  a.W = W;
  hipLaunchKernelGGL((corr_lookup_kernel<4, 4, true>), dim3(f.nblocks), dim3(256), 0, as_stream(stream), a, f);
  return check_launch("raft_convf1_flow");
}
