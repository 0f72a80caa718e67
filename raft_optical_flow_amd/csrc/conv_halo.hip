// Halo-tiled implicit-GEMM convolution for the update block's stride-1
// "same" convs (1x1, 3x3, 1x5, 5x1; core/update.py:6-216), gfx950.
//
// Why a second conv kernel: at one frame pair the update block's GEMMs have
// 7040 rows (55x128 pixels), so a whole conv is a few hundred 64x64 tiles and
// conv_gemm_kernel is bound by the bytes each CU pulls from L2 (every K-step
// re-reads an A tile per tap and a B tile per M-tile), not by the MFMA pipe.
// This kernel cuts those bytes twice over:
//   * A halo: a work-group owns an 8x16 pixel tile; per 32-channel chunk it
//     loads the (8+kh-1) x (16+kw-1) input patch ONCE and runs every tap of
//     the chunk on it (3x3: 180 instead of 9x128 pixel rows);
//   * 128-pixel tiles halve the weight re-reads of the 64-row tiles.
// Both operands move by LDS-DMA (buffer_load ... lds, 1 KiB per wave
// instruction, no VGPR staging), D load sets ahead of the MFMAs, behind a
// counted vmcnt and one raw s_barrier per super-step.
//
// Work-group: 4 waves, one per SIMD; wave w owns tile rows 2w, 2w+1 (32
// pixels) x BNT output channels.  K-step j = (chunk j / T, tap j % T) with
// T = kh*kw; a super-step runs U K-steps.  Inside a wave the K-steps are
// software-pipelined: the LDS fragments of step j+1 are read while the MFMAs
// of step j run and are split to f16 behind them, so one wave per SIMD keeps
// its MFMA pipe fed without a second wave to interleave.
//
// Load set u = K-steps Uu .. Uu+U-1, issued during super-step u - D: every
// wave moves NWP 1-KiB pieces of one K-step's weight block (branch-free:
// K-steps past the end load zeros into their unused ring slot) and, when a
// chunk starts in the set, its share of that chunk's patch.
//
// LDS images (lane-linear DMA writes, XOR-swizzled on the SOURCE address so
// the fragment reads are conflict-free): a patch pixel / weight row is 128 B
// = 8 x 16-B quads; quad q lives in slot q ^ ((x >> 1) & 7), x = the patch
// column (PW is even, so the 16-B bank chunk 8(x&1) + slot is a function of
// x mod 16: the 16 lanes of a ds_read_b128 group read 16 distinct columns)
// or the weight row.
//
// Arithmetic: F16X3 splits each fp32 activation after its LDS read,
// x = hi + lo (hi = f16(x), lo = f16(x - hi), unscaled: the f16-subnormal
// floor of lo is an absolute 2^-25 per element), against the pre-split
// weight (hi, 2048*lo): acc += hi*hi, acl += lo*hi, accx += hi*(2048 lo),
// three independent accumulator chains.  F16 (mixed precision) runs hi*hi;
// BF16 rounds activations and weights to bf16 and runs one
// v_mfma_f32_32x32x16_bf16 product (bf16 mixed precision).
#include <atomic>
#include <type_traits>

#include "conv_common.hpp"

namespace raft {
namespace {

constexpr int HTW = 16;              // tile width (pixels)
constexpr int HTH = 8;               // tile height of the one-round tiles: 128 GEMM rows per work-group
constexpr int HTH_BIG = 16;          // tile height of the multi-round tiles (halo_big): 256 rows
constexpr int HALO_LDS = 160 * 1024;  // LDS per CU (one work-group per CU)

struct HaloArgs {
  raft_conv2d_params p;
  const float* inv_scale;  // big f16x3 tiles: per output column 1 / S_n of the scaled weight (weight_s)
  int K;           // packed weight row length (floats)
  int nch;         // 32-channel chunks
  int nk;          // K-steps = nch * taps
  int gn;          // N-tiles
  int tx_n, ty_n;  // spatial tiles per image
  unsigned w_bytes, in0_bytes, in1_bytes;
};

// One launch runs the tiles of one conv, or of two independent convs of the same shape
// class (raft_conv2d_pair): work-groups [0, grid0) run a[0]'s tiles, the rest a[1]'s.  A work-group
// runs up to m spatial tiles of one N-tile (halo_body): logical work-group g of a conv takes N-tile
// g % gn and spatial tiles (g / gn) * m .. + m-1, so the gn work-groups that share a spatial tile's
// input patch run side by side (and, xcd_tile, on one XCD) as with one tile per work-group.
struct HaloLaunch {
  HaloArgs a[2];
  int sp0, sp1;  // the convs' spatial tiles
  int m;         // spatial tiles per work-group (halo_body)
  int grid0;     // work-groups of a[0] (gn * cdiv(sp0, m))
};

// Smallest patch ring such that chunk c's patch never lands in the slot of a
// chunk that is still read.  In super-steps of U K-steps: chunk c's patch is
// part of load set cT/U, issued during super-step cT/U - D (the prologue's
// sets 0 .. D-1 count as issued before any read); K-step j >= 1 is read
// during super-step (j-1)/U, K-step 0 before super-step 0 (-1).
// late = 1: a K-step's reads may still be in flight one super-step later (the compute waves' relaxed
// barrier wait, halo_body RELAX: the look-ahead reads of the next super-step's first K-step are certified
// at the barrier after it).
constexpr int patch_slots(int T, int U, int D, int late = 0) {
  for (int pa = 1; pa < 16; ++pa) {
    bool ok = true;
    for (int c = pa; c < 512 && ok; ++c) {
      const int last = (c - pa) * T + T - 1;  // last K-step of the slot's previous chunk
      const int rd = last == 0 ? -1 : (last - 1) / U;
      ok = (c * T) / U - D > rd + late;
    }
    if (ok) return pa;
  }
  return 16;
}
constexpr int halo_lds_bytes(int T, int U, int D, int BNT, int PI, int WR) {
  return U * (D + 1) * BNT * WR + patch_slots(T, U, D) * PI * 1024;
}

// WR: bytes per weight row in LDS (128: f16x3 hi | lo; 64: the one-product modes' hi half);
// TH: tile rows (HTH, or HTH_BIG for the multi-round tiles)
template <int KH, int KW, int BNT, int WR = 128, int TH = HTH>
struct HaloCfg {
  static constexpr int T = KH * KW;
  static constexpr int U = (BNT == 32 && T > 1) ? 4 : 2;  // K-steps per super-step
  static constexpr int LB = HALO_LDS;
  static constexpr int PH = TH + KH - 1, PW = HTW + KW - 1, NPIX = PH * PW;
  static constexpr int PI = (NPIX + 7) / 8;  // 1-KiB DMA pieces per patch
  // load sets in flight ahead of the super-step: 3, or 2 where 3 does not fit
#ifdef HALO_D  // dev builds: deeper load rings where they fit
  static constexpr int D = halo_lds_bytes(T, U, HALO_D, BNT, PI, WR) <= LB   ? HALO_D
                           : halo_lds_bytes(T, U, 3, BNT, PI, WR) <= LB ? 3
                                                                              : 2;
#else
  static constexpr int D = halo_lds_bytes(T, U, 3, BNT, PI, WR) <= LB ? 3 : 2;
#endif
  static constexpr int PA = patch_slots(T, U, D);
  // DW: the weight DMAs' lead in super-steps (dev builds: HALO_WX more than the patches' D on the
  // pre-split patch path where the longer weight ring fits)
#ifndef HALO_WX
#define HALO_WX 0
#endif
  static constexpr int DW = (T > 1 && D == 3 && HALO_WX > 0 &&
                             U * (D + HALO_WX + 1) * BNT * WR + PA * PI * 1024 + 16 * 1024 <= LB)
                                ? D + HALO_WX
                                : D;
  static constexpr int SB = U * (DW + 1);  // weight-block ring (K-steps)
  static constexpr int LDS_B = SB * BNT * WR, LDS_A = PA * PI * 1024;
};

#ifdef STAMPS  // dev-only phase timing (tools/conv_bench.py HSTAMPS=1 with a -DSTAMPS variant)
// per compute wave: realtime at entry / exit (100 MHz), then shader cycles of
// the prologue, compute, wait + barrier, epilogue
__device__ unsigned long long g_hstamp[8 * 16384];
__device__ unsigned long long g_lstamp[8 * 16384];  // loader waves (pre-split patch path)
__device__ __forceinline__ unsigned long long hstamp_real() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memrealtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
__device__ __forceinline__ unsigned long long hstamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif

// The tile body: N-tile nt of spatial tiles st0 .. st0 + ntl - 1 of the conv `a` (each a TH x 16-pixel x BNT-column tile;
// smem = the work-group's LDS), one after the other.  With ntl > 1 the K loops of consecutive tiles
// form one stream of super-steps: the loaders run D load sets ahead straight across a tile boundary
// (the next tile's first sets land while the compute waves store the last tile's outputs), so only
// the first tile pays the prologue and the output stores leave in the background of the next tile's
// MFMAs instead of in one burst of every CU at once.  Each tile then runs nkp K-steps, nk rounded up
// to lcm(U, T) so that its chunks start on the patch ring where one tile alone would (the host takes
// ntl > 1 only where that padding is small).  ENC: the encoder features (InstanceNorm partial
// statistics in the epilogue, the input's InstanceNorm applied by the 3x3 loaders); separate
// instantiations, so the update block's convs compile exactly as without them.  TH = HTH_BIG: the
// multi-round tiles (256 pixels x 64 columns, each compute wave 64 x 64 as 2 x 2 MFMA blocks: 2/3
// of the LDS fragment bytes per MFMA and half the weight bytes per pixel of the 128-pixel tiles); in
// f16x3 they run on the column-scaled weight (raft_conv2d_split_weight_scaled: w*S_n = hi + lo, both
// at one scale), so the three products share ONE accumulator chain per block (SC).
constexpr int gcd_c(int a, int b) { return b == 0 ? a : gcd_c(b, a % b); }
// K-steps per tile of a work-group that runs several (see halo_body)
__host__ __device__ inline int halo_nkp(int nk, int U, int T, bool multi) {
  const int l = multi ? U / gcd_c(U, T) * T : U;
  return cdiv(nk, l) * l;
}
template <int KH, int KW, int BNT, int PREC, bool ENC>
constexpr int halo_norm_bytes(int LDS_B, int LDS_A, int D) {
  // the input InstanceNorm tables ({mean, 1/std} per channel) of the images a work-group's tiles
  // cover, in the LDS the rings leave (3x3 split-patch path only)
  return (ENC && KH == 3 && KW == 3 && D == 3) ? ((HALO_LDS - LDS_B - LDS_A) & ~1023) : 0;
}

//
// MT: the multi-tile body (ntl >= 1 at run time).  !MT: exactly one tile per work-group, compiled
// without the tile loop, so the single-round launches (config 2's whole update loop) carry none of
// its cost: no per-load-set tile / chunk divisions, the tile's patch offsets fixed once per lane,
// one K loop and one epilogue (round 4's shared body had made every 128-pixel update conv 7-16 %
// slower in the forward).
// NL: loader waves (4, or 8 for the one-tile f16x3 update convs: RAFT_HALO_NL8, a 768-thread
// work-group whose loaders each issue half the weight DMAs and stage half of each patch)
// KS: compute waves per SIMD (1, or 2 for the K-split form: waves w and w + 4 own the same 32 x 64 block and
// take its even / odd K-steps, each with its own accumulators; the two partial sums meet through LDS in the
// epilogue, where each wave stores half the block's columns -- see halo_ks2)
template <int KH, int KW, int BNT, int PREC, bool ENC = false, int TH = HTH, bool MT = false, int NL = 4, int KS = 1>
__device__ __forceinline__ void halo_body(const HaloArgs* args, int prob, int nt, int st0, int ntl_arg, char* smem) {
  constexpr bool X3 = PREC == RAFT_PREC_F16X3;
  constexpr bool BF = PREC == RAFT_PREC_BF16;
  using C = HaloCfg<KH, KW, BNT, X3 ? 128 : 64, TH>;
  constexpr int T = C::T, U = C::U, D = C::D, PW = C::PW, NPIX = C::NPIX, PI = C::PI, PA = C::PA, SB = C::SB;
  constexpr int DW = C::DW;  // weight lead (== D unless HALO_WX)
  // Weight rows in LDS: f16x3 the packed K-step row as it is (32 hi then 32 lo halves, 128 B);
  // the one-product modes (F16, BF16) read only hi, so only the 64-B hi half of each row
  // moves (half the weight bytes a CU ingests per K-step).  16-B quads XOR-swizzled by row
  // so that the fragment reads are conflict-free: 128-B rows by (row >> 1) & 7, 64-B rows
  // by (row >> 2) & 3.
  constexpr int WROW = X3 ? 128 : 64;          // bytes per weight row in LDS
  constexpr int QPR = WROW / 16;               // 16-B quads per row
  constexpr int RPP = 1024 / WROW;             // rows per 1-KiB DMA piece
  constexpr int NBI = BNT / RPP;    // 1-KiB DMA pieces per weight block (one K-step)
  constexpr int NWP = U * NBI / NL;  // weight pieces per loader wave per load set
  // KSW (KS = 2, dev builds -DHALO_KSW=1): the compute waves issue the weight DMAs (NWPC pieces each per load
  // set) and the loaders stage only the patches.  Measured slower than the loaders issuing both (the DMA issue
  // sits in the compute waves' MFMA stream: profiles/r06b_experiments.txt), so off by default.
#ifndef HALO_KSW
#define HALO_KSW 0
#endif
  constexpr bool KSW = KS > 1 && HALO_KSW;
  constexpr int NWPC = KSW ? U * NBI / (4 * KS) : 1;
  constexpr int LNWP = KSW ? 0 : NWP;  // weight pieces a loader issues per load set
  // Compute waves (32-pixel MFMA row blocks = two tile rows): TH = 8, BNT <= 64: 4 waves along M,
  // each one block (tile rows 2w, 2w+1) x all BNT columns; TH = 8, BNT = 128 (the one-product
  // modes' wide tiles): 2 x 2 waves, each 2 blocks (64 pixels) x 64 columns; TH = 16, BNT = 64:
  // 4 waves along M, each 2 blocks (tile rows 4w .. 4w+3) x 64 columns
  constexpr int WN = BNT == 128 ? 2 : 1;  // compute waves along N
  constexpr int WVM = 4 / WN;             // compute waves along M
  constexpr int MF = TH / 2 / WVM;        // 32-pixel MFMA row blocks per compute wave
  constexpr int WCOL = BNT / WN;          // columns per compute wave
  constexpr int NSUB = WCOL / 32;         // 32-column MFMA subtiles per compute wave
  constexpr bool SC = X3 && TH == HTH_BIG;  // one accumulator on the column-scaled weight
  static_assert(MF >= 1 && MF * WVM * 2 == TH, "tile rows");
  static_assert(!(X3 && MF > 1) || SC, "f16x3 2 x 2 blocks need the one-accumulator (scaled) form");
  static_assert(!ENC || WN == 1, "the InstanceNorm partials are per 32-pixel block of all columns");

  // LSPLIT: the loaders stage each patch through registers and store it
  // pre-split (f16 hi | lo, the weight-row format), so the MFMA waves read
  // ready fragments; 1x1 convs (a patch per K-step, D = 2) keep fp32 patches
  // moved by LDS-DMA and split in the MFMA waves.
#ifndef HALO_NOLSPLIT  // dev builds: the update convs' patches as fp32 by LDS-DMA, split by the compute waves
#define HALO_NOLSPLIT 0
#endif
  constexpr bool LSPLIT = T > 1 && D == 3 && !(HALO_NOLSPLIT && !ENC);
  // SGB: the pre-split path's fragment reads of K-step j+1 pinned into K-step j's MFMA stream, SGB reads
  // per MFMA gap, one K-step per scheduling region.  Left to itself the compiler sinks each read to just
  // before its MFMA and waits lgkmcnt(1) there (the LDS round trip exposed several times per K-step).
  // One read per gap: the update convs -4 % (tools/conv_bench.py, profiles/r06_experiments.txt); two or
  // more per gap, or the encoders' multi-tile bodies, run out of VGPRs at 768 threads and spill.
#ifndef HALO_SGB
#define HALO_SGB 1
#endif
  constexpr int SGB = (ENC && NL == 8) ? 0 : HALO_SGB;
  // RELAX (with SGB's pinned regions): the barrier at the end of a super-step waits only for the reads of
  // its own load sets, not for the look-ahead reads of the next super-step's first K-step issued in its last
  // K-step (lgkmcnt(NRD) instead of lgkmcnt(0): LDS reads complete in order), so the last read's LDS round
  // trip is not exposed at every barrier.  Safe for the weight ring (the next super-step overwrites the slot
  // of the set just finished) and, where patch_slots(.., late = 1) needs no extra slot, for the patch ring.
#ifndef HALO_RELAX
#define HALO_RELAX 1
#endif
  constexpr int NRD1 = NSUB * 2 * (X3 ? 2 : 1) + MF * 2 * (X3 ? 2 : 1);  // LDS reads per K-step
  constexpr bool RELAX = HALO_RELAX && SGB > 0 && LSPLIT && !MT && patch_slots(T, U, D, 1) == PA && NRD1 <= 15;
  static_assert(D >= 2 && C::LDS_B + C::LDS_A <= C::LB, "LDS budget");
  static_assert(KS == 1 || (KS == 2 && !MT && !ENC && LSPLIT && SGB > 0 && MF == 1 && NSUB <= 2 && (NL == 4 || NL == 8) &&
                            SB % 2 == 0 && 8 * 4096 <= C::LDS_B + C::LDS_A && (DW == D || !KSW) && NBI % NWPC == 0 &&
                            NWPC >= 1),
                "the K-split form: one tile of 32 x 64 blocks on the pre-split path, 4 loaders");
  static_assert(NWP >= 1 && NBI % NWP == 0, "a wave's weight pieces lie in one K-step");
  static_assert(U % 2 == 0 && (T == 1 || T >= U), "fragment parity; at most one chunk start per load set");
  constexpr int NORM_BYTES = halo_norm_bytes<KH, KW, BNT, PREC, ENC>(C::LDS_B, C::LDS_A, D);
  static_assert(NORM_BYTES == 0 || NORM_BYTES >= 256 * 8, "room for one image's norm table");

#ifdef STAMPS
  const unsigned long long r_entry = hstamp_real(), c_entry = hstamp_now();
#endif
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  constexpr int NCW = 4 * KS;  // compute waves
  const bool loader = w >= NCW;  // the last NL waves move the operands, the first NCW compute
  const int lw = loader ? w - NCW : w;  // loader index (compute waves: their block index)
  const int wc = w & 3;  // compute waves: block index
  const int kp = KS > 1 ? (w >> 2) & (KS - 1) : 0;  // compute waves: K-step parity (KS = 2)

  const HaloArgs& a = args[prob];
  const raft_conv2d_params& p = a.p;
  const int per = a.tx_n * a.ty_n;
  // tile k of this work-group (N fastest: an output tile's N-tiles share its input patch in L2)
  struct Tile {
    int b, y0, x0, n0, st;
  };
  auto tile_calc = [&](int k) {
    Tile t;
    t.st = st0 + k;
    t.b = t.st / per;
    const int sr = t.st - t.b * per;
    t.y0 = (sr / a.tx_n) * TH;
    t.x0 = (sr % a.tx_n) * HTW;
    t.n0 = nt * BNT;
    return t;
  };
  const Tile tile0 = tile_calc(0);
  auto tile_at = [&](int k) { return MT ? tile_calc(k) : tile0; };
  const int ntl = MT ? ntl_arg : 1;
  const int nk = a.nk, nch = a.nch;
  const int nkp = halo_nkp(nk, U, T, MT && ntl > 1);  // K-steps per tile (multiple of U)
  const int ns_t = nkp / U;                           // super-steps per tile
  const int NS = MT ? ntl * ns_t : ns_t;              // super-steps of the work-group
  const int nchp = nkp / T;                           // patch-ring chunks per tile (ntl > 1: exact)
  // load set u -> (tile kt, set ul within the tile); !MT: (0, u)
  auto set_tile = [&](int u, int& kt, int& ul) {
    if constexpr (MT) {
      kt = u / ns_t;
      ul = u - kt * ns_t;
    } else {
      kt = 0;
      ul = u;
    }
  };
  // patch ring slot of chunk c of tile kt
  auto pslot = [&](int kt, int c) { return MT ? (kt * nchp + c) % PA : c % PA; };

  // Weight pieces of wave lw (a loader, or in the prologue the MFMA wave of the
  // same index): NWP consecutive 8-row pieces of the block of K-step ew of
  // every load set.  Load set u (counted over the work-group's tiles) is set u % ns_t of
  // tile u / ns_t; sets past the last tile load zeros.
  const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(p.weight, a.w_bytes);
  struct WPieces {
    int ew, wpc0;
    unsigned off[NWP];
  };
  auto wpieces = [&](int li) {
    WPieces q;
    q.ew = (li * NWP) / NBI;
    q.wpc0 = (li * NWP) % NBI;
#pragma unroll
    for (int k = 0; k < NWP; ++k) {
      const int r = RPP * (q.wpc0 + k) + lane / QPR;
      const int qd = X3 ? (lane & 7) ^ ((r >> 1) & 7) : (lane & 3) ^ ((r >> 2) & 3);
      // (!MT: the N-tile's first row folded in here; MT: in soff, 0 for the zero sets past the last tile)
      q.off[k] = (unsigned)(r + (MT ? 0 : nt * BNT)) * ((unsigned)a.K * 4u) + (unsigned)qd * 16u;
    }
    return q;
  };
  const WPieces wp0 = wpieces(lw);
  // the compute waves' pieces (KSW): NWPC consecutive pieces of one K-step's block per compute wave
  struct WPiecesC {
    int ew, wpc0;
    unsigned off[NWPC];
  };
  auto wpieces_c = [&](int ci) {
    WPiecesC q;
    q.ew = (ci * NWPC) / NBI;
    q.wpc0 = (ci * NWPC) % NBI;
#pragma unroll
    for (int k = 0; k < NWPC; ++k) {
      const int r = RPP * (q.wpc0 + k) + lane / QPR;
      const int qd = X3 ? (lane & 7) ^ ((r >> 1) & 7) : (lane & 3) ^ ((r >> 2) & 3);
      q.off[k] = (unsigned)(r + nt * BNT) * ((unsigned)a.K * 4u) + (unsigned)qd * 16u;
    }
    return q;
  };
  auto issue_weights_c = [&](int u, const WPiecesC& q) {  // (!MT: load set u of the one tile)
    const int j = U * u + q.ew;
    const bool in = j < nk;
    const int c = j / T, t = j - c * T;
    const unsigned soff = in ? (unsigned)(t * nch + c) * 128u : 0u;
    char* dst = smem + (U * (u % (DW + 1)) + q.ew) * (BNT * WROW) + q.wpc0 * 1024;
#pragma unroll
    for (int k = 0; k < NWPC; ++k) dma16(rs_w, dst + k * 1024, in ? q.off[k] : OFF_INVALID, soff);
  };
  auto issue_weights_q = [&](int u, const WPieces& q) {
    int kt, ul;
    set_tile(u, kt, ul);
    const int j = U * ul + q.ew;
    const bool in = j < nk && (!MT || kt < ntl);
    const int c = j / T, t = j - c * T;
    const int n0 = MT && in ? nt * BNT : 0;
    // packed K-step (tap, chunk) of the tile's N-tile rows
    const unsigned soff = in ? (unsigned)(t * nch + c) * 128u + (unsigned)n0 * ((unsigned)a.K * 4u) : 0u;
    char* dst = smem + (U * (u % (DW + 1)) + q.ew) * (BNT * WROW) + q.wpc0 * 1024;
#pragma unroll
    for (int k = 0; k < NWP; ++k) dma16(rs_w, dst + k * 1024, in ? q.off[k] : OFF_INVALID, soff);
  };
  auto issue_weights = [&](int u) { issue_weights_q(u, wp0); };

  // the input's InstanceNorm (raft_conv2d_params.in_norm: relu((x - mean) / std) applied as the
  // loaders split the patch): the tables of the images of this work-group's tiles into LDS (the
  // host checks that they fit), one barrier for every wave
  float* norm_tab = reinterpret_cast<float*>(smem + C::LDS_B + C::LDS_A);
  int b_first = 0;
  if constexpr (NORM_BYTES > 0) {
    if (p.in_norm) {
      b_first = tile_at(0).b;
      const int nb = tile_at(ntl - 1).b - b_first + 1;
      if (loader)
        for (int i = 64 * lw + lane; i < nb * 2 * p.in0_c; i += 64 * NL)
          norm_tab[i] = p.in_norm[(long)b_first * 2 * p.in0_c + i];
      __syncthreads();
    }
  }

  if (loader) {
#ifdef HALO_LPRIO  // dev builds: the loader waves' issue priority
    __builtin_amdgcn_s_setprio(HALO_LPRIO);
#endif
    // ---- loader waves ------------------------------------------------------
    // (the weights of the prologue's load sets 0 .. D-1 are issued by the MFMA
    // waves, which have nothing else to do then: an LDS-DMA costs its issuing
    // wave 100+ cycles, so the prologue's issue is split over eight waves)
    const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(p.in0, a.in0_bytes);
    const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(p.in1_c ? p.in1 : p.in0, p.in1_c ? a.in1_bytes : a.in0_bytes);
    const int in0_c = p.in0_c, in1_c = p.in1_c;
    const unsigned ld0 = p.in0_ld, ld1 = p.in1_c ? p.in1_ld : p.in0_ld;
    const int in_h = p.in_h, in_w = p.in_w;
    // input pixel of patch pixel pp of tile t, or OFF_INVALID outside the image / patch
    auto patch_pix = [&](const Tile& t, int pp) -> unsigned {
      const int py = pp / PW, px = pp - py * PW;
      const int iy = t.y0 + py - (KH - 1) / 2, ix = t.x0 + px - (KW - 1) / 2;
      const bool ok = pp < NPIX && (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w;
      return ok ? (unsigned)t.b * (unsigned)(in_h * in_w) + (unsigned)iy * (unsigned)in_w + (unsigned)ix : OFF_INVALID;
    };
    // the chunk starting in load set u: its tile kt and chunk c within the tile (at most one: T >= U)
    auto set_chunk = [&](int u, int& kt, int& c) -> bool {
      int ul;
      set_tile(u, kt, ul);
      c = (U * ul + T - 1) / T;
      return (!MT || kt < ntl) && c * T < U * ul + U;
    };
    // Patch pieces of this loader: i = lw, lw+4, ... (< PI), pixels 8i .. 8i+7; per chunk the
    // tile's pixel offsets plus the channel offset
    constexpr int PK = (PI + NL - 1) / NL;
    const int pcw = PI > lw ? (PI - 1 - lw) / NL + 1 : 0;  // this wave's pieces per patch
    // per lane and piece: the channel quad within a chunk (swizzled source) x 4, and (!MT) the
    // input pixel of the one tile, fixed for the work-group
    unsigned pq4[PK], ppix0[PK];
#pragma unroll
    for (int k = 0; k < PK; ++k) {
      const int pp = 8 * (lw + NL * k) + (lane >> 3);
      pq4[k] = 4u * (unsigned)((lane & 7) ^ (((pp % PW) >> 1) & 7));
      ppix0[k] = MT ? 0u : patch_pix(tile0, pp);
    }
    // chunk c of tile kt into patch ring slot pslot(kt, c) (chunks past nch load zeros)
    auto issue_patch = [&](int kt, int c) {
      const Tile t = tile_at(kt);
      const bool s0 = 32 * c < in0_c;  // uniform: the chunk lies in one segment
      const unsigned cb = (unsigned)(s0 ? 32 * c : 32 * c - in0_c);
      const unsigned lim = (unsigned)(s0 ? in0_c : in1_c);
      const unsigned ld = s0 ? ld0 : ld1;
      char* base = smem + C::LDS_B + pslot(kt, c) * (PI * 1024);
#pragma unroll
      for (int k = 0; k < PK; ++k) {
        if (lw + NL * k < PI) {
          const unsigned pix = MT ? patch_pix(t, 8 * (lw + NL * k) + (lane >> 3)) : ppix0[k];
          const unsigned ch = cb + pq4[k];
          const unsigned voff = (pix != OFF_INVALID && ch < lim) ? (pix * ld + ch) * 4u : OFF_INVALID;
          dma16(s0 ? rs0 : rs1, base + (lw + NL * k) * 1024, voff, 0);
        }
      }
    };
    // load set u; returns this wave's DMA count
    auto issue_set = [&](int u, bool weights) -> int {
      int n = 0;
      if (weights) {
        issue_weights(u);
        n = NWP;
      }
      if constexpr (T == 1) {
        int kt, ul;
        set_tile(u, kt, ul);
        if (MT && kt >= ntl) return n;
#pragma unroll
        for (int e = 0; e < U; ++e) issue_patch(kt, U * ul + e);
        return n + U * pcw;
      } else {
        int kt, c;
        if (set_chunk(u, kt, c)) {
          issue_patch(kt, c);
          return n + pcw;
        }
        return n;
      }
    };
    if constexpr (LSPLIT) {
      // 8-channel patch task t = (patch pixel t/4, channel group t%4), NT = 4*NPIX;
      // this wave's tasks t = 64*lw + lane + 64*NL*i.  A chunk's patch is loaded in
      // the super-step that issues its load set and split + stored in the next one
      // (still a super-step before its first read; its slot was free already).
      constexpr int NT = 4 * NPIX, TI = (NT + 64 * NL - 1) / (64 * NL);
      const unsigned tg8 = 8u * (unsigned)(lane & 3);  // channel offset 8g within the chunk (g = t & 3 = lane & 3)
      int tlds[TI];        // byte offset of the task's hi quad in a patch slot (lo: ^ 64), -1 past NT
      unsigned tpix0[TI];  // !MT: the task's input pixel in the one tile (patch_pix)
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        const int t = 64 * lw + lane + 64 * NL * i;
        const int pp = t >> 2, g = t & 3;
        const int px = pp % PW;
        tlds[i] = t < NT ? pp * 128 + ((g ^ ((px >> 1) & 7)) << 4) : -1;
        tpix0[i] = MT ? 0u : patch_pix(tile0, pp);
      }
      auto task_pix = [&](const Tile& tt, int i) {
        return MT ? patch_pix(tt, (64 * lw + lane + 64 * NL * i) >> 2) : tpix0[i];
      };
      using Staged = f32x4[TI][2];
      auto load_patch = [&](int kt, int c, Staged& dst) {  // chunks past the end load zeros
        const Tile tt = tile_at(kt);
        const bool s0 = 32 * c < in0_c;
        const unsigned cb = (unsigned)(s0 ? 32 * c : 32 * c - in0_c);
        const unsigned lim = (unsigned)(s0 ? in0_c : in1_c);
        const unsigned ld = s0 ? ld0 : ld1;
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          const unsigned pix = task_pix(tt, i);
#pragma unroll
          for (int q = 0; q < 2; ++q) {
            const unsigned ch = cb + tg8 + 4u * q;
            const unsigned voff = (pix != OFF_INVALID && ch < lim) ? (pix * ld + ch) * 4u : OFF_INVALID;
            dst[i][q] = buf_load4<0>(s0 ? rs0 : rs1, voff, 0);
          }
        }
      };
      const bool nrm = NORM_BYTES > 0 && p.in_norm != nullptr;
      auto store_patch = [&](int kt, int c, const Staged& src) {
        char* base = smem + C::LDS_B + pslot(kt, c) * (PI * 1024);
        const bool s0 = 32 * c < in0_c;  // (the norm applies to segment 0)
        if (nrm && s0) {
          const Tile tt = tile_at(kt);
          const float2* tab = reinterpret_cast<const float2*>(norm_tab) + (tt.b - b_first) * in0_c;
#pragma unroll
          for (int i = 0; i < TI; ++i) {
            if (tlds[i] >= 0) {
              // channels 32c + 8g .. +7: (x - mean) * rstd, relu; padding (no pixel, or past in0_c) stays 0
              const bool pix_ok = task_pix(tt, i) != OFF_INVALID;
              const int ch = 32 * c + (int)tg8;
              float e[8] = {src[i][0][0], src[i][0][1], src[i][0][2], src[i][0][3],
                            src[i][1][0], src[i][1][1], src[i][1][2], src[i][1][3]};
              if ((in0_c & 7) == 0) {
                // (uniform) the 8 channels' {mean, rstd} as four 16-B reads; a group lies wholly inside
                // or past in0_c
                const bool ok = pix_ok && ch < in0_c;
                const f32x4* t4 = reinterpret_cast<const f32x4*>(tab + (ch < in0_c ? ch : 0));
                const f32x4 q0 = t4[0], q1 = t4[1], q2 = t4[2], q3 = t4[3];
                const float mn[8] = {q0[0], q0[2], q1[0], q1[2], q2[0], q2[2], q3[0], q3[2]};
                const float rs[8] = {q0[1], q0[3], q1[1], q1[3], q2[1], q2[3], q3[1], q3[3]};
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const float v = (e[j] - mn[j]) * rs[j];
                  e[j] = ok ? (p.in_norm_relu ? fmaxf(v, 0.f) : v) : 0.f;
                }
              } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                  const bool ok = pix_ok && ch + j < in0_c;
                  const float2 mr = tab[ok ? ch + j : 0];
                  const float v = (e[j] - mr.x) * mr.y;
                  e[j] = ok ? (p.in_norm_relu ? fmaxf(v, 0.f) : v) : 0.f;
                }
              }
              h8 hi, lo;
              split8<X3, BF>(f32x4{e[0], e[1], e[2], e[3]}, f32x4{e[4], e[5], e[6], e[7]}, hi, lo);
              *reinterpret_cast<h8*>(base + tlds[i]) = hi;
              if constexpr (X3) *reinterpret_cast<h8*>(base + (tlds[i] ^ 64)) = lo;
            }
          }
          return;
        }
#pragma unroll
        for (int i = 0; i < TI; ++i) {
          if (tlds[i] >= 0) {
            h8 hi, lo;
            split8<X3, BF>(src[i][0], src[i][1], hi, lo);
            *reinterpret_cast<h8*>(base + tlds[i]) = hi;
            if constexpr (X3) *reinterpret_cast<h8*>(base + (tlds[i] ^ 64)) = lo;
          }
        }
      };
#ifdef HALO_ABL_PDMA
      // TIMING ABLATION (dev builds only, WRONG results): the patches moved by LDS-DMA as they are in
      // memory (fp32) into the pre-split slots, no register staging and no split -- the bound on what
      // pre-split activation rows in memory would give the loaders (the update convs only)
      if constexpr (!ENC) {
#pragma unroll
        for (int u = 0; u < D; ++u) {
          int kt, c;
          if (set_chunk(u, kt, c)) issue_patch(kt, c);
        }
        wait_vm<0>();
        __builtin_amdgcn_s_barrier();
        for (int s = 0; s < NS; ++s) {
          int nnew = 0;
          if (s + D < NS) {
            int kt, c;
            if (set_chunk(s + D, kt, c)) {
              issue_patch(kt, c);
              nnew += pcw;
            }
            if constexpr (DW == D) {
              issue_weights(s + D);
              nnew += NWP;
            }
          }
          wait_vm_n(s + 1 < NS ? nnew : 0);
          __builtin_amdgcn_s_barrier();
        }
        wait_vm<0>();
        if constexpr (KS > 1) __builtin_amdgcn_s_barrier();
        return;
      }
#endif
      constexpr int PMAX = (U * D + T - 1) / T + 1;  // chunk starts in the prologue's sets
      Staged pv[PMAX];
      int pks[PMAX], pcs[PMAX];
      int nst = 0;
#pragma unroll
      for (int u = 0; u < D; ++u) {
        int kt, c;
        if (set_chunk(u, kt, c)) {
#pragma unroll
          for (int k = 0; k < PMAX; ++k)
            if (k == nst) {
              load_patch(kt, c, pv[k]);
              pks[k] = kt;
              pcs[k] = c;
            }
          ++nst;
        }
      }
      wait_vm<0>();
#pragma unroll
      for (int k = 0; k < PMAX; ++k)
        if (k < nst) store_patch(pks[k], pcs[k], pv[k]);
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the patches are in LDS
      __builtin_amdgcn_s_barrier();
      // Super-step s: store the patch loaded in super-step s-1, load the patch
      // and issue the weights of set s+D, wait until set s+2's weights (issued
      // in s-1) have landed, barrier.
      int pend_k = -1, pend_c = 0;  // chunk staged in pv[0], loaded during the previous super-step
#ifdef STAMPS
      unsigned long long l_st = 0, l_ld = 0, l_w = 0, l_wait = 0, l_bar = 0, l0 = hstamp_now(), l1;
      const unsigned long long l_loop = l0;
#define LSTAMP(acc) (l1 = hstamp_now(), acc += l1 - l0, l0 = l1)
#else
#define LSTAMP(acc)
#endif
      for (int s = 0; s < NS; ++s) {
        if (pend_k >= 0) {
          wait_vm<LNWP>();  // that patch's loads (the weights issued after them may fly on)
          store_patch(pend_k, pend_c, pv[0]);
          pend_k = -1;
        }
        LSTAMP(l_st);
        int nnew = 0;
        if (s + D < NS) {
          int kt, c;
          if (set_chunk(s + D, kt, c)) {
            load_patch(kt, c, pv[0]);
            pend_k = kt;
            pend_c = c;
            nnew = 2 * TI;
          }
          LSTAMP(l_ld);
          // (in the same branch as the patch loads: on every path the compiler sees NWP DMAs behind
          // them, so its own waits for the staged registers stay at vmcnt(NWP), not vmcnt(0))
          if constexpr (DW == D && !KSW) {
#ifndef HALO_ABL_NOW  // TIMING ABLATION (dev builds only, WRONG results): no weight DMAs after the prologue
            issue_weights(s + D);
            nnew += NWP;
#endif
          }
        }
        if constexpr (DW > D && !KSW) {
          if (s + DW < NS) {
            issue_weights(s + DW);
            nnew += NWP;
          }
        }
        LSTAMP(l_w);
        // set s+2 has landed: the weight sets issued in the last DW - D super-steps may fly on
        wait_vm_n(s + 1 < NS ? nnew + (DW - D) * NWP : 0);
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): a patch stored this super-step is in LDS
        LSTAMP(l_wait);
        __builtin_amdgcn_s_barrier();
        LSTAMP(l_bar);
      }
#undef LSTAMP
#ifdef STAMPS
      {  // per loader wave: patch split + store, patch load issue, weight DMA issue, vmcnt wait, barrier, loop total
        const unsigned lid = blockIdx.x * NL + lw;
        if (lane == 0 && lid < 16384) {
          unsigned long long* g = g_lstamp + lid * 8;
          g[0] = l_st;
          g[1] = l_ld;
          g[2] = l_w;
          g[3] = l_wait;
          g[4] = l_bar;
          g[5] = hstamp_now() - l_loop;
          g[6] = 1;
        }
      }
#endif
      wait_vm<0>();
      if constexpr (KS > 1) __builtin_amdgcn_s_barrier();  // (the compute waves' epilogue exchange)
      return;
    }
    // Super-step s: issue load set s+D, wait until load set s+2 has landed
    // (the last K-step of super-step s+1 reads its first block), barrier.
    // hist[k] = this wave's DMA count of the set issued k super-steps ago.
    constexpr int NH = D > 3 ? D - 3 : 1;
    int hist[NH];
    {
      int cnt[D];
#pragma unroll
      for (int u = 0; u < D; ++u) cnt[u] = issue_set(u, false);
      int n = 0;
#pragma unroll
      for (int u = 2; u < D; ++u) n += cnt[u];
      wait_vm_n(n);  // load sets 0 and 1 have landed
#pragma unroll
      for (int k = 0; k < NH; ++k) hist[k] = k < D - 3 ? cnt[D - 1 - k] : 0;
    }
    __builtin_amdgcn_s_barrier();
    for (int s = 0; s < NS; ++s) {
      const int nnew = s + D < NS ? issue_set(s + D, true) : 0;
      int n = D >= 3 ? nnew : 0;  // in flight after set s+2: sets s+3 .. s+D
#pragma unroll
      for (int k = 0; k < D - 3; ++k) n += hist[k];
      wait_vm_n(s + 1 < NS ? n : 0);  // nothing may land after the last barrier
      __builtin_amdgcn_s_barrier();  // set s+2 readable by every wave
#pragma unroll
      for (int k = NH - 1; k > 0; --k) hist[k] = hist[k - 1];
      hist[0] = nnew;
    }
    wait_vm<0>();  // nothing may land after the work-group exits
    return;
  }

  // ---- compute waves: fragments --------------------------------------------
  const int m = lane & 31, h = lane >> 5;
  const int wm = wc % WVM, cb = (wc / WVM) * WCOL;  // the wave's pixel blocks and first column
  int ppbase[MF];  // patch pixel of this lane's row in block f (tap 0, 0)
#pragma unroll
  for (int f = 0; f < MF; ++f) ppbase[f] = (2 * (wm * MF + f) + (m >> 4)) * PW + (m & 15);
  const int bsw = X3 ? (m >> 1) & 7 : (m >> 2) & 3;  // swizzle of weight row cb + sb*32 + m
  // accx: the hi * (2048 lo) chain of the unscaled f16x3 form (not used by SC or one-product modes)
  constexpr int AXF = X3 && !SC ? MF : 1, AXS = X3 && !SC ? NSUB : 1;
  f32x16 acc[MF][NSUB], accx[AXF][AXS];
  auto clear_acc = [&]() {
#pragma unroll
    for (int f = 0; f < MF; ++f)
#pragma unroll
      for (int sb = 0; sb < NSUB; ++sb) acc[f][sb] = f32x16{};
#pragma unroll
    for (int f = 0; f < AXF; ++f)
#pragma unroll
      for (int sb = 0; sb < AXS; ++sb) accx[f][sb] = f32x16{};
  };
  clear_acc();
  // Fragment reads run ahead of the MFMAs: the B fragments of K-step j+1 and
  // the A (activation) values of K-step j+2 are read while K-step j's MFMAs
  // run, and A of j+1 (read one K-step earlier) is split to f16 behind them,
  // so neither the LDS latency nor the split stalls the MFMA stream.
  // B cursor: the weight ring slot of the next K-step to read; A cursor:
  // (tap, ky, kx) and the patch ring slot of the next K-step to read.
  int b_bs = kp;  // (KS = 2: the odd waves start at K-step 1)
  int a_t = 0, a_ky = 0, a_kx = 0, a_ps = 0;
  struct Frag {
    h8 ah[MF][2], al[MF][2];
    h8 bh[NSUB][2], bl[NSUB][2];
  };
  f32x4 av[MF][4];  // raw A values of the K-step after the next
  auto read_b = [&](Frag& F) {
    const char* Bb = smem + b_bs * (BNT * WROW);
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        F.bh[sb][qq] = *reinterpret_cast<const h8*>(Bb + (cb + sb * 32 + m) * WROW + (((2 * h + qq) ^ bsw) << 4));
        if constexpr (X3)
          F.bl[sb][qq] = *reinterpret_cast<const h8*>(Bb + (cb + sb * 32 + m) * WROW + (((4 + 2 * h + qq) ^ bsw) << 4));
      }
    }
    b_bs = b_bs + KS >= SB ? b_bs + KS - SB : b_bs + KS;  // (KS = 2: this wave's next K-step)
  };
  auto advance_a = [&]() {
    ++a_kx;
    if (a_kx == KW) {
      a_kx = 0;
      ++a_ky;
    }
    if (++a_t == T) {
      a_t = 0;
      a_ky = 0;
      a_ps = a_ps + 1 == PA ? 0 : a_ps + 1;
    }
  };
  auto read_a = [&]() {
    const char* Ab = smem + C::LDS_B + a_ps * (PI * 1024);
    const int sw = (((m & 15) + a_kx) >> 1) & 7;  // swizzle of patch column px
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const int pp = ppbase[f] + (a_ky * PW + a_kx);
#pragma unroll
      for (int jq = 0; jq < 4; ++jq)
        av[f][jq] = *reinterpret_cast<const f32x4*>(Ab + pp * 128 + (((4 * h + jq) ^ sw) << 4));
    }
    advance_a();
  };
  auto read_a_split = [&](Frag& F) {  // LSPLIT: the patch holds f16 hi | lo quads
    const char* Ab = smem + C::LDS_B + a_ps * (PI * 1024);
    const int sw = (((m & 15) + a_kx) >> 1) & 7;
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      const char* row = Ab + (ppbase[f] + (a_ky * PW + a_kx)) * 128;
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        F.ah[f][qq] = *reinterpret_cast<const h8*>(row + (((2 * h + qq) ^ sw) << 4));
        if constexpr (X3) F.al[f][qq] = *reinterpret_cast<const h8*>(row + (((4 + 2 * h + qq) ^ sw) << 4));
      }
    }
#pragma unroll
    for (int k = 0; k < KS; ++k) advance_a();
  };
  auto split_a = [&](Frag& F) {
#pragma unroll
    for (int f = 0; f < MF; ++f) {
#ifdef HALO_ABL_NOSPLIT  // timing ablation (dev builds only): bit casts instead of the split
      F.ah[f][0] = __builtin_bit_cast(h8, av[f][0]);
      F.al[f][0] = __builtin_bit_cast(h8, av[f][1]);
      F.ah[f][1] = __builtin_bit_cast(h8, av[f][2]);
      F.al[f][1] = __builtin_bit_cast(h8, av[f][3]);
#else
      split8<X3, BF>(av[f][0], av[f][1], F.ah[f][0], F.al[f][0]);
      split8<X3, BF>(av[f][2], av[f][3], F.ah[f][1], F.al[f][1]);
#endif
    }
  };
  // the MFMAs of one accumulator never follow each other back to back
  auto mfma_step = [&](const Frag& F) {
#pragma unroll
    for (int qq = 0; qq < 2; ++qq) {
      if constexpr (BF) {
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb)
            acc[f][sb] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(
                __builtin_bit_cast(bf8, F.ah[f][qq]), __builtin_bit_cast(bf8, F.bh[sb][qq]), acc[f][sb], 0, 0, 0);
      } else {
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb)
            acc[f][sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[f][qq], F.bh[sb][qq], acc[f][sb], 0, 0, 0);
      }
      if constexpr (SC) {  // hi * lo and lo * hi at the scale of hi * hi: the same chain
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb)
            acc[f][sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[f][qq], F.bl[sb][qq], acc[f][sb], 0, 0, 0);
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb)
            acc[f][sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.al[f][qq], F.bh[sb][qq], acc[f][sb], 0, 0, 0);
      } else if constexpr (X3) {
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb)
            accx[f][sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.ah[f][qq], F.bl[sb][qq], accx[f][sb], 0, 0, 0);
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb)
            acc[f][sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(F.al[f][qq], F.bh[sb][qq], acc[f][sb], 0, 0, 0);
      }
    }
  };
  // the fragments of a tile's first K-step (its K-step 0 is the next to read)
  Frag F[2];
  auto first_frags = [&]() {
    if constexpr (LSPLIT) {
      read_b(F[0]);
      read_a_split(F[0]);
    } else {
      read_a();
      read_b(F[0]);
      split_a(F[0]);
      read_a();
    }
  };
  // the tile's outputs (register r of block f holds row m = (r&3) + 8(r>>2) + 4h of its 32 pixels)
  auto epilogue = [&](const Tile& t) {
    if constexpr (SC) {  // undo the column scale S_n (a power of two: exact)
#pragma unroll
      for (int sb = 0; sb < NSUB; ++sb) {
        const float is = a.inv_scale[t.n0 + cb + sb * 32 + m];
#pragma unroll
        for (int f = 0; f < MF; ++f)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[f][sb][r] *= is;
      }
    } else if constexpr (X3) {
#pragma unroll
      for (int f = 0; f < MF; ++f)
#pragma unroll
        for (int sb = 0; sb < NSUB; ++sb)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[f][sb][r] += accx[f][sb][r] * (1.0f / SPLIT_SCALE);
    }
    f32x4 stv[NSUB];  // ENC: the wave's InstanceNorm partials per column (its MF blocks combined)
    // the output geometry read once (the kernel argument sits at a run-time offset, prob: read inside
    // the row loop it was a scalar load and wait per row), rows by selects, not branches
    const int oh = __builtin_amdgcn_readfirstlane(p.out_h), ow = __builtin_amdgcn_readfirstlane(p.out_w);
    const int rowb = t.b * oh;
#pragma unroll
    for (int f = 0; f < MF; ++f) {
      int rows[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int y = t.y0 + 2 * (wm * MF + f) + (mm >> 4), x = t.x0 + (mm & 15);
        rows[r] = ((y < oh) & (x < ow)) ? (rowb + y) * ow + x : -1;
      }
#pragma unroll
      for (int sb = 0; sb < NSUB; ++sb) tile_epilogue<false>(p, rows, t.n0 + cb + sb * 32 + m, acc[f][sb]);
      if constexpr (ENC) {
        if (p.stats_part) {  // InstanceNorm partials of the raw output, per wave (slot: spatial tile x 4 + wave)
#pragma unroll
          for (int sb = 0; sb < NSUB; ++sb) {
            const int n = t.n0 + sb * 32 + m;
            const f32x4 v = tile_stats_vals(rows, acc[f][sb], p.bias ? p.bias[n < p.n ? n : 0] : 0.f);
            stv[sb] = f == 0 ? v : stats_combine(stv[sb], v);
            if (f == MF - 1) stats_write(p, n, (long)t.st * 4 + w, stv[sb]);
          }
        }
      }
    }
  };

  // KS = 2: the even and odd waves of a block hold partial sums of all its outputs.  Each keeps one half (64
  // columns: even waves columns 0-31, odd 32-63; 32 columns: even waves the block's first tile row, odd the
  // second), hands the other half to its partner through LDS (the operand rings are free by now: <= 4 KiB per
  // wave) and stores its half: the block's epilogue runs on both waves of the SIMD.  The sum even + odd is one
  // fp32 addition per element (commutative: the same bits on either wave).
  auto epilogue_ks2 = [&](const Tile& t) {
    if constexpr (KS > 1 && NSUB == 1) {
      if constexpr (X3 && !SC) {
#pragma unroll
        for (int r = 0; r < 16; ++r) acc[0][0][r] += accx[0][0][r] * (1.0f / SPLIT_SCALE);
      }
      // rows r < 8: the first tile row of the block (m < 16); r >= 8 the second
      f32x4* mine = reinterpret_cast<f32x4*>(smem + (wc * 2 + kp) * 4096) + lane * 2;
      const f32x4* theirs = reinterpret_cast<const f32x4*>(smem + (wc * 2 + (kp ^ 1)) * 4096) + lane * 2;
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        f32x4 v;
#pragma unroll
        for (int i = 0; i < 4; ++i) v[i] = kp ? acc[0][0][4 * q + i] : acc[0][0][8 + 4 * q + i];
        mine[q ^ (lane & 1)] = v;
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();  // (the loaders join it on their way out)
      f32x16 keep = acc[0][0];
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const f32x4 o = theirs[q ^ (lane & 1)];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
          if (kp)
            keep[8 + 4 * q + i] += o[i];
          else
            keep[4 * q + i] += o[i];
        }
      }
      const int oh = __builtin_amdgcn_readfirstlane(p.out_h), ow = __builtin_amdgcn_readfirstlane(p.out_w);
      const int rowb = t.b * oh;
      int rows[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int y = t.y0 + 2 * wm + (mm >> 4), x = t.x0 + (mm & 15);
        rows[r] = ((y < oh) & (x < ow)) ? (rowb + y) * ow + x : -1;
      }
      if (kp)
        tile_epilogue<false, 8, 8>(p, rows, t.n0 + cb + m, keep);
      else
        tile_epilogue<false, 0, 8>(p, rows, t.n0 + cb + m, keep);
    } else if constexpr (KS > 1) {
      if constexpr (X3 && !SC) {
#pragma unroll
        for (int sb = 0; sb < NSUB; ++sb)
#pragma unroll
          for (int r = 0; r < 16; ++r) acc[0][sb][r] += accx[0][sb][r] * (1.0f / SPLIT_SCALE);
      }
      f32x16 keep, send;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        keep[r] = kp ? acc[0][1][r] : acc[0][0][r];
        send[r] = kp ? acc[0][0][r] : acc[0][1][r];
      }
      // LDS slot of wave (wc, kp): 64 lanes x 64 B, the lane's four 16-B quads rotated by lane & 3
      f32x4* mine = reinterpret_cast<f32x4*>(smem + (wc * 2 + kp) * 4096) + lane * 4;
      const f32x4* theirs = reinterpret_cast<const f32x4*>(smem + (wc * 2 + (kp ^ 1)) * 4096) + lane * 4;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        mine[q ^ (lane & 3)] = f32x4{send[4 * q], send[4 * q + 1], send[4 * q + 2], send[4 * q + 3]};
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();  // (the loaders join it on their way out)
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const f32x4 o = theirs[q ^ (lane & 3)];
#pragma unroll
        for (int i = 0; i < 4; ++i) keep[4 * q + i] += o[i];
      }
      const int oh = __builtin_amdgcn_readfirstlane(p.out_h), ow = __builtin_amdgcn_readfirstlane(p.out_w);
      const int rowb = t.b * oh;
      int rows[16];
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
        const int y = t.y0 + 2 * wm + (mm >> 4), x = t.x0 + (mm & 15);
        rows[r] = ((y < oh) & (x < ow)) ? (rowb + y) * ow + x : -1;
      }
      tile_epilogue<false>(p, rows, t.n0 + cb + kp * 32 + m, keep);
    }
  };

  // ---- compute waves: pipeline ---------------------------------------------
  // Super-step s runs K-steps Us .. Us+U-1 (its reads reach K-step U(s+1)+1,
  // all in load sets s and s+1), then one barrier.  K-steps past nk (up to
  // nkp) run on zero weights and zero patches: they add exact zeros, and the
  // loop body has no branches.  A tile's last super-step reads nothing ahead
  // (the next tile's first fragments are read after its epilogue).
  if constexpr (KS > 1) {
    if (kp) advance_a();  // the odd waves' first K-step is K-step 1
  }
  const WPiecesC wpc = wpieces_c(KSW ? w : 0);
  if constexpr (KSW) {  // every compute wave issues its pieces of sets 0 .. D-1 (and later of every set)
#pragma unroll
    for (int u = 0; u < DW; ++u) issue_weights_c(u, wpc);
    wait_vm<NWPC * (DW - 2)>();
  } else if constexpr (KS > 1) {  // compute wave w issues the prologue pieces of loader w (4 loaders: the even waves)
    if (NL == 8 || kp == 0) {
#pragma unroll
      for (int u = 0; u < DW; ++u) issue_weights(u);
      wait_vm<NWP * (DW - 2)>();
    }
  } else if constexpr (NL == 8) {  // (each compute wave also issues the prologue pieces of loader lw + 4)
    const WPieces wp1 = wpieces(lw + 4);
#pragma unroll
    for (int u = 0; u < DW; ++u) {
      issue_weights(u);
      issue_weights_q(u, wp1);
    }
    wait_vm<2 * NWP * (DW - 2)>();  // the weights of sets 0 and 1
  } else {
#pragma unroll
    for (int u = 0; u < DW; ++u) issue_weights(u);
    wait_vm<NWP * (DW - 2)>();
  }      // the weights of sets 0 and 1 (sets 2 .. D-1: before the first loop barrier)
  __builtin_amdgcn_s_barrier();  // load sets 0 and 1 have landed
#ifdef HALO_PRIO
  __builtin_amdgcn_s_setprio(HALO_PRIO);
#endif
  // SB1 (KS = 2, dev builds -DHALO_KS2_SB1=1): one fragment buffer per compute wave (each K-step's fragments
  // read at its start; the partner wave's MFMAs cover the LDS round trip), for the 128 VGPRs of 1024-thread
  // work-groups
#ifndef HALO_KS2_SB1
#define HALO_KS2_SB1 0
#endif
  constexpr bool SB1 = KS > 1 && HALO_KS2_SB1;
  if constexpr (!SB1) first_frags();
#ifdef STAMPS
  unsigned long long t_cmp = 0, t_wait = 0, t_bar = 0, t_epi = 0, t0 = hstamp_now();
  const unsigned long long c_loop = t0;
#endif
  // one K-step on the pre-split path: the fragments of this wave's next K-step into nxt while the
  // MFMAs run on cur (SGB: the reads pinned one per MFMA gap, one scheduling region per K-step)
  auto kstep_split = [&](Frag& nxt, const Frag& cur) {
    if constexpr (SGB > 0) __builtin_amdgcn_sched_barrier(0);
    read_b(nxt);
    read_a_split(nxt);
    mfma_step(cur);
    if constexpr (SGB > 0) {
      constexpr int NRD = NRD1;
      constexpr int NMF = 2 * MF * NSUB * (X3 ? 3 : 1);
      constexpr int RPG = SGB;
      constexpr int NG = NRD / RPG < NMF ? NRD / RPG : NMF;  // full read groups
      constexpr int REM = NRD - NG * RPG;                     // the rest, in slot NG (or NMF - 1)
#pragma unroll
      for (int i = 0; i < NMF; ++i) {
        if (i < NG) __builtin_amdgcn_sched_group_barrier(0x100, RPG, 0);
        if constexpr (REM > 0) {
          if (i == (NG < NMF ? NG : NMF - 1)) __builtin_amdgcn_sched_group_barrier(0x100, REM, 0);
        }
        __builtin_amdgcn_sched_group_barrier(0x8, 1, 0);
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  };
  // KS = 2: this wave's U / 2 K-steps of a super-step; PAR: the fragment buffer of its first (the
  // buffers alternate per own K-step, so with one own K-step per super-step the loop runs in pairs)
  int nnew_c = 0;  // KSW: weight pieces this wave issued in the current super-step
  auto superstep_ks = [&](auto par_tag, int s) {
    constexpr int PAR = decltype(par_tag)::value;
    nnew_c = 0;
    if constexpr (KSW) {
      if (s + D < NS) {
        issue_weights_c(s + D, wpc);
        nnew_c = NWPC;
      }
    }
#pragma unroll
    for (int e = 0; e < U / KS; ++e) {
      if constexpr (SB1) {
        __builtin_amdgcn_sched_barrier(0);
        read_b(F[0]);
        read_a_split(F[0]);
        mfma_step(F[0]);
        __builtin_amdgcn_sched_barrier(0);
      } else {
        kstep_split(F[(PAR + e + 1) & 1], F[(PAR + e) & 1]);
      }
    }
  };
  // one super-step's K-steps; LAST: the tile's last super-step, which reads nothing ahead
  auto superstep = [&](auto last_tag) {
    constexpr bool LAST = decltype(last_tag)::value;
#pragma unroll
    for (int e = 0; e < U; ++e) {
#ifdef HALO_ABL_MFMAONLY  // timing ablation (dev builds only): MFMAs on fragments read once
      mfma_step(F[e & 1]);
      asm volatile("" ::"v"(F[0].ah[0][0]), "v"(F[1].ah[0][0]));
#else
      if (LAST && e == U - 1) {
        mfma_step(F[e & 1]);
      } else if constexpr (LSPLIT) {
        kstep_split(F[(e + 1) & 1], F[e & 1]);
      } else {
        read_b(F[(e + 1) & 1]);
        mfma_step(F[e & 1]);
        split_a(F[(e + 1) & 1]);
        read_a();
      }
#endif
    }
  };
  bool first = true;
  auto step_end = [&]() {
#ifdef STAMPS
    unsigned long long t2 = hstamp_now();
    t_cmp += t2 - t0;
#endif
    if constexpr (RELAX)
      __builtin_amdgcn_s_waitcnt(0xC07F | (NRD1 << 8));  // lgkmcnt(NRD1): all but the look-ahead reads
    else
      __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the next fragments are in registers
    if constexpr (KSW) {
      wait_vm_n(nnew_c);  // this wave's pieces of every set but the one issued in this super-step have landed
    } else {
      if (first) wait_vm<0>();  // the prologue's weight sets 2 .. D-1 (this wave's only DMAs)
    }
    first = false;
#ifdef STAMPS
    unsigned long long t3 = hstamp_now();
    t_wait += t3 - t2;
#endif
    __builtin_amdgcn_s_barrier();  // the reads of super-step s are done; set s+2 has landed
#ifdef STAMPS
    t0 = hstamp_now();
    t_bar += t0 - t3;
#endif
  };
  if constexpr (KS > 1) {
    using P0 = std::integral_constant<int, 0>;
    using P1 = std::integral_constant<int, 1>;
    int s = 0;
    if constexpr ((U / KS) % 2 == 1) {
      for (; s + 1 < NS; s += 2) {
        superstep_ks(P0{}, s);
        step_end();
        superstep_ks(P1{}, s + 1);
        step_end();
      }
    }
    for (; s < NS; ++s) {
      superstep_ks(P0{}, s);
      step_end();
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // (the last look-ahead reads, before the ring is reused)
    __builtin_amdgcn_sched_barrier(0);
    epilogue_ks2(tile0);
#ifdef STAMPS
    const unsigned long long t4 = hstamp_now();
    t_epi += t4 - t0;
#endif
  } else if constexpr (!MT) {
    // one tile: the last super-step's look-ahead reads land in ring slots nobody writes any more
    for (int s = 0; s < NS; ++s) {
      superstep(std::false_type{});
      step_end();
    }
    if constexpr (RELAX) __builtin_amdgcn_s_waitcnt(0xC07F);  // (the last look-ahead reads, before exit)
    __builtin_amdgcn_sched_barrier(0);
    epilogue(tile0);
#ifdef STAMPS
    const unsigned long long t4 = hstamp_now();
    t_epi += t4 - t0;
#endif
  } else {
  for (int kt = 0; kt < ntl; ++kt) {
    for (int sl = 0; sl + 1 < ns_t; ++sl) {
      superstep(std::false_type{});
      step_end();
    }
    superstep(std::true_type{});
    step_end();
    // (non-LSPLIT: av already holds the next tile's K-step 0, read one K-step ahead)
    __builtin_amdgcn_sched_barrier(0);
    epilogue(tile_at(kt));
    clear_acc();
    __builtin_amdgcn_sched_barrier(0);
    // the next tile's first fragments (after the last tile: reads of ring slots nobody uses,
    // unconditional so that no path keeps the old fragments live through the epilogue)
    if constexpr (LSPLIT) {
      read_b(F[0]);
      read_a_split(F[0]);
    } else {
      read_b(F[0]);
      split_a(F[0]);
      read_a();
    }
#ifdef STAMPS
    const unsigned long long t4 = hstamp_now();
    t_epi += t4 - t0;
    t0 = t4;
#endif
  }
  }
#ifdef STAMPS
  {
    const unsigned long long c_exit = hstamp_now(), r_exit = hstamp_real();
    const unsigned wid = blockIdx.x * NCW + w;
    if (lane == 0 && wid < 16384) {
      unsigned long long* g = g_hstamp + wid * 8;
      g[0] = r_entry;
      g[1] = r_exit;
      g[2] = c_loop - c_entry;
      g[3] = t_cmp;
      g[4] = t_wait + t_bar;
      g[5] = t_epi;
      g[6] = c_exit - c_entry;
    }
  }
#endif
}

// One conv (or an independent pair, raft_conv2d_pair) per launch: work-group g runs tiles
// N-tile g % gn of spatial tiles (g / gn) * m .. + m-1 of its conv (the pair's first grid0
// work-groups take a[0]'s tiles).
template <int KH, int KW, int BNT, int PREC, bool ENC = false, int TH = HTH, bool MT = false, int NL = 4, int KS = 1>
__global__ __launch_bounds__(64 * (4 * KS + NL)) void conv_halo_kernel(HaloLaunch hl) {
  using C = HaloCfg<KH, KW, BNT, PREC == RAFT_PREC_F16X3 ? 128 : 64, TH>;
  constexpr int NORM_BYTES = halo_norm_bytes<KH, KW, BNT, PREC, ENC>(C::LDS_B, C::LDS_A, C::D);
  __shared__ __attribute__((aligned(1024))) char smem[C::LDS_B + C::LDS_A + NORM_BYTES];
  int g = xcd_tile(blockIdx.x, gridDim.x);
  const int prob = g >= hl.grid0 ? 1 : 0;
  g -= prob * hl.grid0;
  const int gn = hl.a[prob].gn;
  if constexpr (MT) {
    const int st0 = (g / gn) * hl.m;
    const int ntl = min(hl.m, (prob ? hl.sp1 : hl.sp0) - st0);
    halo_body<KH, KW, BNT, PREC, ENC, TH, true, NL>(hl.a, prob, g % gn, st0, ntl, smem);
  } else {  // (hl.m == 1)
    halo_body<KH, KW, BNT, PREC, ENC, TH, false, NL, KS>(hl.a, prob, g % gn, g / gn, 1, smem);
  }
}

// the kernel of a launch: the multi-tile body where the plan runs several tiles per work-group
// (l.m > 1), else the one-tile body.  (The one-product 3x3 wide tiles never run several:
// halo_mt_ok.)
// the one-tile f16x3 update convs' loader waves: 8, or 4 (RAFT_HALO_NL8=0; raft_conv2d_set_halo_loaders)
std::atomic<int> g_halo_nl{0};  // 0: from the environment
bool halo_nl8() {
  int v = g_halo_nl.load(std::memory_order_relaxed);
  if (v == 0) {
    // (default 8: config 2 +1.0-1.4 % in three interleaved pairs on one box, profiles/r05e_experiments.txt)
    const char* e = getenv("RAFT_HALO_NL8");
    v = e && e[0] == '0' ? 4 : 8;
    g_halo_nl.store(v, std::memory_order_relaxed);
  }
  return v == 8;
}
#ifndef HALO_KS2_NL8
#define HALO_KS2_NL8 0
#endif
#ifndef HALO_KS2_BN32  // dev builds: the K-split form for the 32-column update convs too (measured slower: their
#define HALO_KS2_BN32 0  // 4 K-steps per super-step leave the 4 loaders further behind, profiles/r06b_experiments.txt)
#endif
// the K-split form (two compute waves per SIMD, halo_body KS = 2) for the one-tile f16x3 update convs with
// 64-column tiles (default; RAFT_HALO_KS2=0 or raft_conv2d_set_halo_ks(1): one compute wave per SIMD).
// Config 2, bench.py interleaved on one box: 144.7 / 143.9 / 144.2 -> 146.9 / 147.0 / 147.0 pairs/s, the
// iteration's update convs 151-153 -> 146-148 us (profiles/r06b_experiments.txt)
std::atomic<int> g_halo_ks{0};  // 0: from the environment
bool halo_ks2() {
  int v = g_halo_ks.load(std::memory_order_relaxed);
  if (v == 0) {
    const char* e = getenv("RAFT_HALO_KS2");
    v = e && e[0] == '0' ? 1 : 2;
    g_halo_ks.store(v, std::memory_order_relaxed);
  }
  return v == 2;
}
bool halo_nl8_enc() {
  // (default on: config 2 +0.1 / +0.3 % in two interleaved pairs on one box, profiles/r05f_experiments.txt;
  // read per launch so that a test can switch it -- a plan captures the launches it made)
  const char* e = getenv("RAFT_HALO_NL8_ENC");
  return !(e && e[0] == '0');
}
// the shapes compiled without the multi-tile body (launch_halo_mt): halo_mt_ok never plans m > 1 for
// them, and the launch refuses m > 1 (the one-tile kernel would run only 1/m of the spatial tiles)
constexpr bool halo_no_mt(int prec, int taps, int bn) { return prec != RAFT_PREC_F16X3 && taps == 9 && bn == 128; }

template <int KH, int KW, int BNT, int PREC, bool ENC = false, int TH = HTH>
void launch_halo_mt(const HaloLaunch& l, dim3 grid, hipStream_t s) {
  constexpr bool NO_MT = halo_no_mt(PREC, KH * KW, BNT);
  if (NO_MT && l.m > 1) {
    fprintf(stderr, "raft_hip: internal error: a one-tile-only halo conv was planned with %d tiles per work-group\n", l.m);
    abort();
  }
  // the 8-loader form: one-tile f16x3 update-block convs (default; RAFT_HALO_NL8=0: 4 loaders)
  constexpr bool CAN_NL8 = PREC == RAFT_PREC_F16X3 && !ENC && TH == HTH && BNT <= 64 && KH * KW > 1;
  // and for the encoders' f16x3 3x3 convs on 128-pixel tiles (default; RAFT_HALO_NL8_ENC=0: 4): their loaders also
  // apply the input InstanceNorm
  constexpr bool CAN_NL8E = PREC == RAFT_PREC_F16X3 && ENC && TH == HTH && BNT <= 64 && KH * KW == 9;
  if constexpr (CAN_NL8E) {
    if (halo_nl8_enc()) {
      if (l.m > 1)
        hipLaunchKernelGGL((conv_halo_kernel<KH, KW, BNT, PREC, ENC, TH, true, 8>), grid, dim3(768), 0, s, l);
      else
        hipLaunchKernelGGL((conv_halo_kernel<KH, KW, BNT, PREC, ENC, TH, false, 8>), grid, dim3(768), 0, s, l);
      return;
    }
  }
  // the K-split form: the one-tile f16x3 update convs with 64-column tiles on the pre-split path
  constexpr bool CAN_KS2 = CAN_NL8 && (BNT == 64 || (BNT == 32 && HALO_KS2_BN32)) &&
                           HaloCfg<KH, KW, BNT, 128, TH>::D == 3 && !HALO_NOLSPLIT;
  if (!NO_MT && l.m > 1) {
    hipLaunchKernelGGL((conv_halo_kernel<KH, KW, BNT, PREC, ENC, TH, !NO_MT>), grid, dim3(512), 0, s, l);
  } else {
    if constexpr (CAN_KS2) {
      if (halo_ks2()) {
#if HALO_KS2_NL8  // dev builds: 8 loaders beside the 8 compute waves (1024 threads, 128 VGPRs per wave)
        hipLaunchKernelGGL((conv_halo_kernel<KH, KW, BNT, PREC, ENC, TH, false, 8, 2>), grid, dim3(1024), 0, s, l);
#else
        hipLaunchKernelGGL((conv_halo_kernel<KH, KW, BNT, PREC, ENC, TH, false, 4, 2>), grid, dim3(768), 0, s, l);
#endif
        return;
      }
    }
    if constexpr (CAN_NL8) {
      if (halo_nl8()) {
        hipLaunchKernelGGL((conv_halo_kernel<KH, KW, BNT, PREC, ENC, TH, false, 8>), grid, dim3(768), 0, s, l);
        return;
      }
    }
    hipLaunchKernelGGL((conv_halo_kernel<KH, KW, BNT, PREC, ENC, TH, false>), grid, dim3(512), 0, s, l);
  }
}

template <int KH, int KW, int PREC>
void launch_halo_p(const HaloLaunch& l, int bn, int th, dim3 grid, hipStream_t s) {
  const raft_conv2d_params& p = l.a[0].p;
  if constexpr (KH == 3 && KW == 3) {
    if (th == HTH_BIG) {  // (halo_pick: N tile 64)
      if (p.stats_part || p.in_norm)
        launch_halo_mt<3, 3, 64, PREC, true, HTH_BIG>(l, grid, s);
      else
        launch_halo_mt<3, 3, 64, PREC, false, HTH_BIG>(l, grid, s);
      return;
    }
  } else if constexpr (KH * KW == 5) {
    // 1x5 / 5x1 big tiles: the one-product modes' 64-B weight rows leave LDS for the three pre-split
    // 16 x 20 patches the T = 5 ring needs (D = 3); f16x3's 128-B rows do not, so it runs D = 2 with
    // fp32 patches split by the compute waves (216 / 232 VGPRs)
    if (th == HTH_BIG) {
      launch_halo_mt<KH, KW, 64, PREC, false, HTH_BIG>(l, grid, s);
      return;
    }
  }
  if constexpr (PREC != RAFT_PREC_F16X3) {
    if (bn == 128) {  // (conv_halo_launch picks it only without stats_part / in_norm)
      launch_halo_mt<KH, KW, 128, PREC>(l, grid, s);
      return;
    }
  }
  if constexpr ((KH == 1 && KW == 1) || (KH == 3 && KW == 3)) {
    if (p.stats_part || p.in_norm) {  // (one conv per launch: raft_conv2d_pair takes neither)
      if (bn == 64)
        launch_halo_mt<KH, KW, 64, PREC, true>(l, grid, s);
      else
        launch_halo_mt<KH, KW, 32, PREC, true>(l, grid, s);
      return;
    }
  }
  if (bn == 64)
    launch_halo_mt<KH, KW, 64, PREC>(l, grid, s);
  else
    launch_halo_mt<KH, KW, 32, PREC>(l, grid, s);
}
template <int KH, int KW>
void launch_halo_k(const HaloLaunch& l, int bn, int th, dim3 grid, hipStream_t s) {
  const int prec = l.a[0].p.precision;
  if (prec == RAFT_PREC_F16X3)
    launch_halo_p<KH, KW, RAFT_PREC_F16X3>(l, bn, th, grid, s);
  else if (prec == RAFT_PREC_BF16)
    launch_halo_p<KH, KW, RAFT_PREC_BF16>(l, bn, th, grid, s);
  else
    launch_halo_p<KH, KW, RAFT_PREC_F16>(l, bn, th, grid, s);
}

bool halo_enabled() {
  static const bool enabled = [] {
    const char* e = getenv("RAFT_CONV_HALO");
    return !(e && e[0] == '0');
  }();
  return enabled;
}

// The halo kernel's view of a conv it covers (stride 1, "same" padding, 1x1 / 3x3 / 1x5 /
// 5x1, VEC mode, split-weight precisions), all but the N-tile width; false otherwise.
bool halo_problem(const HaloOperands& o, HaloArgs& a) {
  const raft_conv2d_params& p = o.p;
  if (p.mode != RAFT_CONV_VEC || p.stride_h != 1 || p.stride_w != 1) return false;
  if (p.precision != RAFT_PREC_F16X3 && p.precision != RAFT_PREC_F16 && p.precision != RAFT_PREC_BF16) return false;
  const int kh = p.kh, kw = p.kw;
  const bool shape = (kh == 1 && kw == 1) || (kh == 3 && kw == 3) || (kh == 1 && kw == 5) || (kh == 5 && kw == 1);
  if (!shape || p.pad_h != (kh - 1) / 2 || p.pad_w != (kw - 1) / 2) return false;
  if (p.out_h != p.in_h || p.out_w != p.in_w || p.n <= 4) return false;
  a.p = p;
  a.inv_scale = nullptr;
  a.K = o.k_pad;
  a.nch = o.k_pad / (kh * kw) / 32;
  a.nk = a.nch * kh * kw;
  a.tx_n = cdiv(p.out_w, HTW);
  a.ty_n = cdiv(p.out_h, HTH);
  a.w_bytes = o.w_bytes;
  a.in0_bytes = o.in0_bytes;
  a.in1_bytes = o.in1_bytes;
  a.gn = 0;
  return true;
}

long halo_spatial(const HaloArgs& a) { return (long)a.p.batch * a.tx_n * a.ty_n; }

// The big tiles (TH = HTH_BIG, N tile 64) for 3x3 / 1x5 / 5x1 convs.  A big tile does the work of two
// 128-pixel tiles at ~0.85-0.9 of their cost per pixel (the K loop runs closer to the MFMA rate, but
// its prologue and the epilogue's store burst are twice as long), and every launch runs in whole
// rounds of one work-group per CU, so the choice counts rounds: big tiles iff
//   ceil(T_big / CUs) * RAFT_HALO_BIG_COST (1.8 = 2 x 0.9) < ceil(T_128 / CUs)
// (tools/conv_bench.py on one box: convc2 at B=8 156.5 vs 175.1 us, 3 vs 6 rounds; fh1 at B=8
// 116.1 vs 112.9 us, 4 vs 7 rounds; config 5's bf16 convs with 3 vs 4 and 2 vs 2 rounds 34 %
// slower as big tiles).  RAFT_HALO_BIG_MIN=0 turns them off (default 1: no other floor).
// f16x3 needs the scaled weight (raft_conv2d_params.weight_s).
long halo_big_min() {
  static const long v = [] {
    const char* e = getenv("RAFT_HALO_BIG_MIN");
    return e ? atol(e) : 1L;
  }();
  return v;
}
double halo_big_cost() {
  static const double v = [] {
    const char* e = getenv("RAFT_HALO_BIG_COST");
    return e ? atof(e) : 1.8;
  }();
  return v;
}
// the CU count of the device the launch runs on (the current device), cached per device: the tile
// choice (rounds rule, tiles per work-group) follows it when one process drives several GPUs
long halo_cus() {
  constexpr int MAXDEV = 64;
  static std::atomic<int> cache[MAXDEV];  // 0 = not queried yet
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess) return 256L;
  if (dev >= 0 && dev < MAXDEV) {
    const int c = cache[dev].load(std::memory_order_relaxed);
    if (c > 0) return (long)c;
  }
  int cus = 0;
  if (hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || cus <= 0) cus = 256;
  if (dev >= 0 && dev < MAXDEV) cache[dev].store(cus, std::memory_order_relaxed);
  return (long)cus;
}
bool halo_big_ok(const HaloOperands& o) {
  const raft_conv2d_params& p = o.p;
  if (o.n_pad % 64) return false;
  if (p.kh == 3 && p.kw == 3) return p.precision != RAFT_PREC_F16X3 || p.weight_s != nullptr;
  // 1x5 / 5x1: no encoder features (launch_halo_p)
  return p.kh * p.kw == 5 && (p.precision != RAFT_PREC_F16X3 || p.weight_s != nullptr) && !p.stats_part && !p.in_norm;
}
long halo_big_tiles(const HaloOperands& o) {
  const raft_conv2d_params& p = o.p;
  return (long)p.batch * cdiv(p.out_h, HTH_BIG) * cdiv(p.out_w, HTW) * (o.n_pad / 64);
}
long halo_small_tiles(const HaloOperands& o) {  // 128-pixel x 64-column tiles
  const raft_conv2d_params& p = o.p;
  return (long)p.batch * cdiv(p.out_h, HTH) * cdiv(p.out_w, HTW) * (o.n_pad / 64);
}
// the rounds rule above for a launch of big_tiles vs small_tiles work-groups
bool halo_big_pays(long big_tiles, long small_tiles) {
  const long mn = halo_big_min(), cus = halo_cus();
  if (mn <= 0 || big_tiles < mn) return false;
  return (double)cdiv_l(big_tiles, cus) * halo_big_cost() < (double)cdiv_l(small_tiles, cus);
}
// the least multi-tile plan cost of the conv on tiles of th rows (halo_plan_grid's cost, in tile times
// of that size), below
double halo_mt_plan_cost(const HaloOperands& o, int th);
// RAFT_HALO_BIG_MT=1: where the rounds rule keeps the 128-pixel tiles, also compare the two tile sizes'
// multi-tile plans (a launch with rounds to spare runs several tiles per work-group, so whole rounds are
// not the unit there): big tiles when cost(big) * RAFT_HALO_BIG_COST < cost(128-pixel)
bool halo_big_mt() {
  static const bool v = [] {
    const char* e = getenv("RAFT_HALO_BIG_MT");
    return e && e[0] == '1';
  }();
  return v;
}
// Tile rows of a conv's launch: HTH_BIG where the big tiles qualify and pay, and (the one-product
// modes without encoder features) the 128-column tiles do not apply
int halo_pick_th(const HaloOperands& o, bool wide) {
  if (wide || !halo_big_ok(o)) return HTH;
  if (halo_big_pays(halo_big_tiles(o), halo_small_tiles(o))) return HTH_BIG;
  if (halo_big_mt() && halo_big_min() > 0 && halo_big_tiles(o) >= halo_big_min() &&
      halo_mt_plan_cost(o, HTH_BIG) * halo_big_cost() < halo_mt_plan_cost(o, HTH))
    return HTH_BIG;
  return HTH;
}
// the big tiles' operands: spatial tiles of TH_BIG rows; f16x3 reads the scaled weight
void halo_set_th(const HaloOperands& o, HaloArgs& a, int th) {
  a.ty_n = cdiv(a.p.out_h, th);
  if (th == HTH_BIG && a.p.precision == RAFT_PREC_F16X3) {
    a.p.weight = reinterpret_cast<const float*>(o.p.weight_s);
    a.inv_scale = reinterpret_cast<const float*>(reinterpret_cast<const char*>(o.p.weight_s) + (size_t)o.w_bytes);
  }
}

// LDS left for the input-norm tables of a 3x3 ENC instantiation (halo_norm_bytes)
template <int BNT, int WR, int TH>
long halo_norm_cap_t() {
  using C = HaloCfg<3, 3, BNT, WR, TH>;
  return halo_norm_bytes<3, 3, BNT, RAFT_PREC_F16X3, true>(C::LDS_B, C::LDS_A, C::D);
}
long halo_norm_cap(int bn, int prec, int th) {
  const bool x3 = prec == RAFT_PREC_F16X3;
  if (th == HTH_BIG) return x3 ? halo_norm_cap_t<64, 128, HTH_BIG>() : halo_norm_cap_t<64, 64, HTH_BIG>();
  if (bn == 64) return x3 ? halo_norm_cap_t<64, 128, HTH>() : halo_norm_cap_t<64, 64, HTH>();
  return x3 ? halo_norm_cap_t<32, 128, HTH>() : halo_norm_cap_t<32, 64, HTH>();
}

// Tiles per work-group (halo_body): a launch with more tiles than CUs may run m spatial tiles per
// work-group, the m of least cost in tile times (below), where padding every tile's K loop to
// lcm(U, T) K-steps costs at most 1/8 and the input-norm tables of the images a work-group covers
// fit its LDS; otherwise one tile per work-group.  RAFT_HALO_MT=0: always one.
bool halo_mt_enabled() {
  static const bool enabled = [] {
    const char* e = getenv("RAFT_HALO_MT");
    return !(e && e[0] == '0');
  }();
  return enabled;
}
double halo_mt_cost() {
  static const double v = [] {
    const char* e = getenv("RAFT_HALO_MT_COST");
    return e ? atof(e) : 0.8;
  }();
  return v;
}
bool halo_mt_ok(const HaloArgs& a, int bn, int th, long m) {
  const int T = a.p.kh * a.p.kw, U = (bn == 32 && T > 1) ? 4 : 2;
  // measured (profiles/r04mt3_experiments.txt, config 5's update convs at 135x240): the one-product
  // modes' 3x3 convs with several N-tiles ran 18-30 % slower on multi-tile work-groups (their short
  // K loops do not cover the next tile's loads beside the last one's stores); their 1x1 / 1x5 convs
  // and every f16x3 conv gained
  if (halo_no_mt(a.p.precision, T, bn)) return false;  // (not compiled: wide tiles unmeasured)
  if (a.p.precision != RAFT_PREC_F16X3 && T == 9 && a.gn > 1) return false;
  const int n1 = halo_nkp(a.nk, U, T, false), nm = halo_nkp(a.nk, U, T, true);
  if ((long)(nm - n1) * 8 > n1) return false;
  if (a.p.in_norm) {
    const long per_img = (long)a.tx_n * a.ty_n;
    const long imgs = cdiv_l(m, per_img) + 1;
    if (imgs * a.p.in0_c * 8 > halo_norm_cap(bn, a.p.precision, th)) return false;
  }
  return true;
}
// sets l.m (spatial tiles per work-group) and l.grid0 for the launch of l.a[0] (and l.a[1] of a
// pair, pair = true); returns the grid size (cost_out: the plan's cost in tile times)
long halo_plan_grid(HaloLaunch& l, int bn, int th, bool pair, double* cost_out = nullptr) {
  const long cus = halo_cus();
  const long s0 = halo_spatial(l.a[0]), s1 = pair ? halo_spatial(l.a[1]) : 0;
  const long g0 = l.a[0].gn, g1 = pair ? l.a[1].gn : 0;
  auto wgs = [&](long m) { return g0 * cdiv_l(s0, m) + g1 * cdiv_l(s1, m); };
  // cost in tile times: rounds of work-groups x (the first tile + RAFT_HALO_MT_COST per later tile:
  // the prologue and the output stores of the later tiles run under the K loops)
  long m = 1;
  double best = (double)cdiv_l(wgs(1), cus);
  if (halo_mt_enabled() && wgs(1) > cus) {
    const double f = halo_mt_cost();
    for (long c = 2; c <= 64; ++c) {
      const double cost = (double)cdiv_l(wgs(c), cus) * (1.0 + f * (double)(c - 1));
      if (cost < best && halo_mt_ok(l.a[0], bn, th, c) && (!pair || halo_mt_ok(l.a[1], bn, th, c))) {
        best = cost;
        m = c;
      }
    }
  }
  l.m = (int)m;
  l.sp0 = (int)s0;
  l.sp1 = (int)s1;
  l.grid0 = (int)(g0 * cdiv_l(s0, m));
  if (cost_out) *cost_out = best;
  return wgs(m);
}

double halo_mt_plan_cost(const HaloOperands& o, int th) {
  HaloLaunch l;
  if (!halo_problem(o, l.a[0])) return 1e30;
  halo_set_th(o, l.a[0], th);
  const int bn = th == HTH_BIG ? 64 : halo_spatial(l.a[0]) * (o.n_pad / 64) > 128 ? 64 : 32;
  l.a[0].gn = o.n_pad / bn;
  l.a[1] = l.a[0];
  double cost = 1e30;
  halo_plan_grid(l, bn, th, false, &cost);
  return cost;
}

void launch_halo(const HaloLaunch& l, int bn, int th, long wgs, hipStream_t s) {
  const raft_conv2d_params& p = l.a[0].p;
  dim3 grid((unsigned)wgs);
  if (p.kh == 1 && p.kw == 1)
    launch_halo_k<1, 1>(l, bn, th, grid, s);
  else if (p.kh == 3)
    launch_halo_k<3, 3>(l, bn, th, grid, s);
  else if (p.kh == 1)
    launch_halo_k<1, 5>(l, bn, th, grid, s);
  else
    launch_halo_k<5, 1>(l, bn, th, grid, s);
}


}  // namespace

#ifdef STAMPS
extern "C" int raft_debug_hstamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hstamp), sizeof(unsigned long long) * (size_t)n);
}
extern "C" int raft_debug_lstamps(unsigned long long* host, int n, int clear) {
  if (clear) {
    static unsigned long long zero[8 * 16384];
    return (int)hipMemcpyToSymbol(HIP_SYMBOL(g_lstamp), zero, sizeof(zero));
  }
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_lstamp), sizeof(unsigned long long) * (size_t)n);
}
#endif

// the loader-wave count of the one-tile f16x3 update-block convs (4 or 8); returns the previous
extern "C" int raft_conv2d_set_halo_loaders(int nl) {
  const int prev = halo_nl8() ? 8 : 4;
  if (nl == 4 || nl == 8) g_halo_nl.store(nl, std::memory_order_relaxed);
  return prev;
}

// the compute waves per SIMD of the one-tile f16x3 update convs with 64-column tiles (1 or 2); returns the
// previous
extern "C" int raft_conv2d_set_halo_ks(int ks) {
  const int prev = halo_ks2() ? 2 : 1;
  if (ks == 1 || ks == 2) g_halo_ks.store(ks, std::memory_order_relaxed);
  return prev;
}

// whether the conv takes its input InstanceNorm in the loaders (raft_conv2d_params.in_norm): the
// 3x3 convs' split-patch path (D = 3 for both N-tile widths), <= 256 input channels
bool conv_halo_norm_ok(const HaloOperands& o) {
  HaloArgs a;
  if (!halo_enabled() || !halo_problem(o, a)) return false;
  const raft_conv2d_params& p = o.p;
  return p.kh == 3 && p.kw == 3 && p.in0_c <= 256 && HaloCfg<3, 3, 64>::D == 3 && HaloCfg<3, 3, 32>::D == 3;
}

// the least 128-column tile count for the wide tiles (RAFT_HALO_WIDE_MIN): 256, one round (512 until
// r04j: config 5's bf16 update convs 364 -> 351 us per iteration, 47.0 -> 47.8 pairs/s on one box)
long halo_wide_min() {
  static const long v = [] {
    const char* e = getenv("RAFT_HALO_WIDE_MIN");
    return e ? atol(e) : 256L;
  }();
  return v;
}
bool halo_wide_enabled() {
  static const bool enabled = [] {
    const char* e = getenv("RAFT_HALO_WIDE");
    return !(e && e[0] == '0');
  }();
  return enabled;
}

// The tile of a conv: the one-product modes' 128-column tiles (wide) where at least two rounds of
// them remain (512), else the big tiles where the rounds rule picks them, else the wide tiles from
// RAFT_HALO_WIDE_MIN (256) of them, else the 128-pixel tiles.  Returns the tile rows; `wide` out.
int halo_pick(const HaloOperands& o, const HaloArgs& a, bool& wide) {
  const raft_conv2d_params& p = o.p;
  const bool can = p.precision != RAFT_PREC_F16X3 && !p.stats_part && !p.in_norm && o.n_pad % 128 == 0 &&
                   halo_wide_enabled();
  const long n = halo_spatial(a) * (o.n_pad / 128);
  wide = can && n >= 512;
  const int th = halo_pick_th(o, wide);
  if (!wide && th != HTH_BIG) wide = can && n >= halo_wide_min();
  return th;
}

// tile rows conv_halo_launch picks for the conv (HTH or HTH_BIG), 0 when the halo kernel does not run it
int conv_halo_tile_rows(const HaloOperands& o) {
  HaloArgs a;
  if (!halo_enabled() || !halo_problem(o, a)) return 0;
  bool wide;
  return halo_pick(o, a, wide);
}

bool conv_halo_covers(const HaloOperands& o) {
  HaloArgs a;
  return halo_enabled() && halo_problem(o, a);
}

int conv_halo_stats_slots(const HaloOperands& o) {
  HaloArgs a;
  if (!halo_enabled() || !halo_problem(o, a)) return 0;
  // only the ENC instantiations (1x1 and 3x3, launch_halo_p) write InstanceNorm partials: one slot
  // per compute wave of a spatial tile (the tile rows of conv_halo_launch's pick)
  if (!((o.p.kh == 1 && o.p.kw == 1) || (o.p.kh == 3 && o.p.kw == 3))) return 0;
  const int th = halo_pick_th(o, false);  // (ENC convs never take the 128-column tiles)
  return a.tx_n * cdiv(o.p.out_h, th) * 4;
}

// the launch of one conv: operands, N-tile width, tile rows and grid size; false when the halo
// kernel does not cover the conv
static bool halo_plan(const HaloOperands& o, HaloLaunch& l, int& bn, int& th, long& wgs) {
  if (!halo_enabled() || !halo_problem(o, l.a[0])) return false;
  const long spatial = halo_spatial(l.a[0]);
  // one work-group per CU (LDS): 64 output channels per work-group unless
  // 32 still fits the grid in one round of 256 CUs with half of them idle at 64;
  // the one-product modes take 128-column tiles (2 x 2 waves of 64 x 64) by halo_pick
  // (RAFT_HALO_WIDE=0: never)
  bool wide;
  th = halo_pick(o, l.a[0], wide);
  bn = th == HTH_BIG ? 64 : wide ? 128 : spatial * (o.n_pad / 64) > 128 ? 64 : 32;
  halo_set_th(o, l.a[0], th);
  l.a[0].gn = o.n_pad / bn;
  const long tiles = halo_spatial(l.a[0]) * l.a[0].gn;
  if (tiles >= (1L << 31)) return false;
  l.a[1] = l.a[0];
  wgs = halo_plan_grid(l, bn, th, false);
  return true;
}

// tiles per work-group of the conv's halo launch (halo_body), 0 when the halo kernel does not run it
int conv_halo_tiles_per_wg(const HaloOperands& o) {
  HaloLaunch l;
  int bn, th;
  long wgs;
  return halo_plan(o, l, bn, th, wgs) ? l.m : 0;
}

// Launches the halo kernel when the conv is one it covers; returns 1 without launching
// otherwise.  Arguments are already validated by raft_conv2d.
int conv_halo_launch(const HaloOperands& o, hipStream_t s) {
  HaloLaunch l;
  int bn, th;
  long wgs;
  if (!halo_plan(o, l, bn, th, wgs)) return 1;
  launch_halo(l, bn, th, wgs, s);
  return 0;
}

// Two independent convs of one shape class and precision in one launch (their tiles side
// by side in the grid, one N-tile width for both); returns 1 without launching when the
// pair does not qualify.
int conv_halo_launch_pair(const HaloOperands& o0, const HaloOperands& o1, hipStream_t s) {
  HaloLaunch l;
  if (!halo_enabled() || !halo_problem(o0, l.a[0]) || !halo_problem(o1, l.a[1])) return 1;
  const raft_conv2d_params &p0 = o0.p, &p1 = o1.p;
  if (p0.kh != p1.kh || p0.kw != p1.kw || p0.precision != p1.precision) return 1;
  // each conv's own tile rows (the rounds rule, as raft_conv2d would pick them): the big f16x3 tiles
  // run the scaled one-chain arithmetic, so only convs that pick the same rows share a launch, which
  // keeps the pair bit-identical to the two single launches (raft_hip.h); otherwise they run in order
  const int th = halo_pick_th(o0, false);
  if (halo_pick_th(o1, false) != th) return 1;
  halo_set_th(o0, l.a[0], th);
  halo_set_th(o1, l.a[1], th);
  const long s0 = halo_spatial(l.a[0]), s1 = halo_spatial(l.a[1]);
  const int bn = th == HTH_BIG ? 64 : s0 * (o0.n_pad / 64) + s1 * (o1.n_pad / 64) > 128 ? 64 : 32;
  if (o0.n_pad % bn || o1.n_pad % bn) return 1;
  l.a[0].gn = o0.n_pad / bn;
  l.a[1].gn = o1.n_pad / bn;
  const long t0 = s0 * l.a[0].gn, tiles = t0 + s1 * l.a[1].gn;
  if (tiles >= (1L << 31)) return 1;
  launch_halo(l, bn, th, halo_plan_grid(l, bn, th, true), s);
  return 0;
}


}  // namespace raft
