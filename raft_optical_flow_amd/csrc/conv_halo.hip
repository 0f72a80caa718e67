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
// instruction, no VGPR staging), so D super-steps of loads stay in flight
// behind a counted vmcnt and a raw s_barrier.
//
// Work-group: 8 waves = 2 K-groups x 4 waves.  K-step j = (chunk j / T, tap
// j % T), T = kh*kw; super-step s runs K-step 2s in group 0 and 2s+1 in group
// 1 (two waves per SIMD interleave), each wave a 32-pixel x BNT-channel block
// (two tile rows).  The groups' accumulators are summed through LDS.
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
// weight (hi, 2048*lo):  acc += hi*hi + lo*hi,  accx += hi*(2048 lo).
// F16 (mixed precision) runs hi*hi only.
#include "conv_common.hpp"

namespace raft {
namespace {

constexpr int HTW = 16;  // tile width (pixels)
constexpr int HTH = 8;   // tile height: 128 GEMM rows per work-group

struct HaloArgs {
  raft_conv2d_params p;
  int K;           // packed weight row length (floats)
  int nch;         // 32-channel chunks
  int nk;          // K-steps = nch * taps
  int gn;          // N-tiles
  int tx_n, ty_n;  // spatial tiles per image
  unsigned w_bytes, in0_bytes, in1_bytes;
};

// Smallest number of patch slots such that chunk c's patch, issued with the
// loads of super-step floor(cT/2) at super-step floor(cT/2) - D, never lands
// in the slot of a chunk still read at or after that issue point (a K-step's
// fragments are read one super-step before its MFMAs).
template <int T, int D>
constexpr int patch_slots() {
  for (int pa = 1; pa < 16; ++pa) {
    bool ok = true;
    for (int c = pa; c < 256; ++c)
      if ((c * T) / 2 - D < ((c - pa) * T + T - 1) / 2) ok = false;
    if (ok) return pa;
  }
  return 16;
}

#ifdef STAMPS  // dev-only phase timing (tools/conv_bench.py HSTAMPS=1 with a -DSTAMPS variant)
__device__ unsigned long long g_hstamp[4 * 16384];
__device__ __forceinline__ unsigned long long hstamp_now() {
  unsigned long long t;
  __builtin_amdgcn_sched_barrier(0);
  asm volatile("s_memtime %0\n\ts_waitcnt lgkmcnt(0)" : "=s"(t)::"memory");
  __builtin_amdgcn_sched_barrier(0);
  return t;
}
#endif

__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, void* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// s_waitcnt vmcnt(n) only (expcnt / lgkmcnt at their maxima); n <= 15 here
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | 0x70 | 0xF00 | ((N >> 4) << 14));
}
__device__ __forceinline__ void wait_vm_n(int n) {
  switch (n) {
    case 0: wait_vm<0>(); break;
    case 1: wait_vm<1>(); break;
    case 2: wait_vm<2>(); break;
    case 3: wait_vm<3>(); break;
    case 4: wait_vm<4>(); break;
    case 5: wait_vm<5>(); break;
    case 6: wait_vm<6>(); break;
    case 7: wait_vm<7>(); break;
    case 8: wait_vm<8>(); break;
    case 9: wait_vm<9>(); break;
    case 10: wait_vm<10>(); break;
    case 11: wait_vm<11>(); break;
    case 12: wait_vm<12>(); break;
    case 13: wait_vm<13>(); break;
    case 14: wait_vm<14>(); break;
    default: wait_vm<15>(); break;
  }
}

// x - f16 half of hpk, exact in fp32 (v_fma_mix: the f16 operand widened in the ALU)
__device__ __forceinline__ float sub_half_lo(unsigned hpk, float x) {
  float r;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hpk), "v"(x));
  return r;
}
__device__ __forceinline__ float sub_half_hi(unsigned hpk, float x) {
  float r;
  asm("v_fma_mix_f32 %0, %1, -1.0, %2 op_sel:[1,0,0] op_sel_hi:[1,0,0]" : "=v"(r) : "v"(hpk), "v"(x));
  return r;
}

using f2 = __attribute__((ext_vector_type(2))) float;
using h2 = __attribute__((ext_vector_type(2))) _Float16;

// 8 floats -> 8 f16 hi (+ 8 f16 lo = f16(x - hi)) : 4 VALU per 2 elements
template <bool LO>
__device__ __forceinline__ void split8(const f32x4 x0, const f32x4 x1, h8& hi, h8& lo) {
  const float v[8] = {x0[0], x0[1], x0[2], x0[3], x1[0], x1[1], x1[2], x1[3]};
  unsigned hp[4], lp[4];
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const h2 h = __builtin_convertvector((f2){v[2 * e], v[2 * e + 1]}, h2);
    hp[e] = __builtin_bit_cast(unsigned, h);
    if constexpr (LO) {
      const float d0 = sub_half_lo(hp[e], v[2 * e]);
      const float d1 = sub_half_hi(hp[e], v[2 * e + 1]);
      lp[e] = __builtin_bit_cast(unsigned, __builtin_convertvector((f2){d0, d1}, h2));
    }
  }
  hi = __builtin_bit_cast(h8, (__attribute__((ext_vector_type(4))) unsigned){hp[0], hp[1], hp[2], hp[3]});
  if constexpr (LO)
    lo = __builtin_bit_cast(h8, (__attribute__((ext_vector_type(4))) unsigned){lp[0], lp[1], lp[2], lp[3]});
}

template <int KH, int KW, int BNT, int PREC>
__global__ __launch_bounds__(512, 1) void conv_halo_kernel(HaloArgs a) {
  constexpr int T = KH * KW;
#ifdef HALO_D  // dev builds: load depth override
  constexpr int D = T == 1 ? 3 : HALO_D;
#else
  constexpr int D = T == 1 ? 3 : 4;             // load sets issued ahead of the super-step
#endif
  constexpr int PH = HTH + KH - 1, PW = HTW + KW - 1, NPIX = PH * PW;
  constexpr int PI = (NPIX + 7) / 8;            // 1-KiB DMA pieces per patch
  constexpr int PA = patch_slots<T, D>();
  constexpr int SB = 2 * D;                     // weight-block ring (K-steps)
  constexpr int NBI = BNT / 8;                  // DMA pieces per weight block
  constexpr int NSUB = BNT / 32;                // 32-column MFMA subtiles per wave
  constexpr int LDS_B = SB * BNT * 128;
  constexpr int LDS_A = PA * PI * 1024;
  constexpr bool X3 = PREC == RAFT_PREC_F16X3;
  static_assert(LDS_B + LDS_A <= 160 * 1024, "LDS budget");
  static_assert(NSUB * 16 * 256 * 4 <= LDS_B + LDS_A, "K-group reduction buffer");
  __shared__ __attribute__((aligned(1024))) char smem[LDS_B + LDS_A];

  const raft_conv2d_params& p = a.p;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const int g = w >> 2, wm = w & 3;

  // tile (N fastest: an output tile's N-tiles share its input patch in L2)
  const int q = xcd_tile(blockIdx.x, gridDim.x);
  const int nt = q % a.gn, st = q / a.gn;
  const int per = a.tx_n * a.ty_n;
  const int b = st / per, sr = st - b * per;
  const int y0 = (sr / a.tx_n) * HTH, x0 = (sr % a.tx_n) * HTW;
  const int n0 = nt * BNT;
  const int nk = a.nk, nch = a.nch;
  const int ns = (nk + 1) >> 1;

  const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(p.weight, a.w_bytes);
  const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(p.in0, a.in0_bytes);
  const __amdgpu_buffer_rsrc_t rs1 = make_rsrc(p.in1_c ? p.in1 : p.in0, p.in1_c ? a.in1_bytes : a.in0_bytes);
  const int in0_c = p.in0_c, in1_c = p.in1_c;
  const unsigned ld0 = p.in0_ld, ld1 = p.in1_c ? p.in1_ld : p.in0_ld;
  const int in_h = p.in_h, in_w = p.in_w;
  const unsigned pb = (unsigned)b * (unsigned)(in_h * in_w);
  const unsigned wrow = (unsigned)a.K * 4u;

  // ---- loads ---------------------------------------------------------------
  // Everything per lane is fixed by the tile, so the DMA addresses are
  // precomputed once; per K-step only scalar offsets change (the main loop
  // must stay light on SALU: eight waves share one scalar unit).
  // Patch pieces of this wave: i = w, w+8, w+16 (< PI): pixels 8i .. 8i+7.
  constexpr int PK = (PI + 7) / 8;
  unsigned ppix[PK];  // input pixel index, or OFF_INVALID outside the image / patch
  unsigned pq4[PK];   // the lane's channel quad within a chunk (swizzled source), x 4
#pragma unroll
  for (int k = 0; k < PK; ++k) {
    const int pp = 8 * (w + 8 * k) + (lane >> 3);
    const int py = pp / PW, px = pp - py * PW;
    const int qd = (lane & 7) ^ ((px >> 1) & 7);
    const int iy = y0 + py - (KH - 1) / 2, ix = x0 + px - (KW - 1) / 2;
    const bool ok = pp < NPIX && (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w;
    ppix[k] = ok ? pb + (unsigned)iy * (unsigned)in_w + (unsigned)ix : OFF_INVALID;
    pq4[k] = 4u * (unsigned)qd;
  }
  const int pcw = PI > w ? (PI - 1 - w) / 8 + 1 : 0;  // this wave's pieces per patch
  auto issue_patch = [&](int c, int slot) {
    const bool s0 = 32 * c < in0_c;  // uniform: the chunk lies in one segment
    const unsigned cb = (unsigned)(s0 ? 32 * c : 32 * c - in0_c);
    const unsigned lim = (unsigned)(s0 ? in0_c : in1_c);
    const unsigned ld = s0 ? ld0 : ld1;
    char* base = smem + LDS_B + slot * (PI * 1024);
#pragma unroll
    for (int k = 0; k < PK; ++k) {
      if (w + 8 * k < PI) {
        const unsigned ch = cb + pq4[k];
        const unsigned voff = (ppix[k] != OFF_INVALID && ch < lim) ? (ppix[k] * ld + ch) * 4u : OFF_INVALID;
        dma16(s0 ? rs0 : rs1, base + (w + 8 * k) * 1024, voff, 0);
      }
    }
  };
  // Weight pieces: rows 8i .. 8i+7 of a K-step's BNT-row block; wave w loads
  // piece w of both K-steps of a super-step (BNT = 64) or piece w%4 of K-step
  // w/4 (BNT = 32)
  const int wpiece = NBI == 8 ? w : (w & 3);
  unsigned wvoff;
  {
    const int r = 8 * wpiece + (lane >> 3);
    const int qd = (lane & 7) ^ ((r >> 1) & 7);
    wvoff = (unsigned)(n0 + r) * wrow + (unsigned)qd * 16u;
  }
  // issue cursor: the next K-step to load, as (chunk, tap), its K-step
  // index in the packed weight (tap*nch + chunk) and its ring slots
  int i_j = 0, i_c = 0, i_t = 0, i_kk = 0, i_bs = 0, i_ps = 0;
  auto issue_set = [&]() {  // load set of the next super-step; returns this wave's DMA count
    int n = 0;
#pragma unroll
    for (int e = 0; e < 2; ++e) {
      if (i_j < nk) {
        if (i_t == 0) {
          issue_patch(i_c, i_ps);
          n += pcw;
        }
        if (NBI == 8 || (w >> 2) == e) {
          dma16(rs_w, smem + i_bs * (BNT * 128) + wpiece * 1024, wvoff, (unsigned)i_kk * 128u);
          ++n;
        }
        ++i_j;
        ++i_t;
        i_kk += nch;
        i_bs = i_bs + 1 == SB ? 0 : i_bs + 1;
        if (i_t == T) {
          i_t = 0;
          ++i_c;
          i_kk = i_c;
          i_ps = i_ps + 1 == PA ? 0 : i_ps + 1;
        }
      }
    }
    return n;
  };

  // ---- fragments -----------------------------------------------------------
  const int m = lane & 31, h = lane >> 5;
  const int ppbase = (2 * wm + (m >> 4)) * PW + (m & 15);
  int bro[NSUB];  // the lane's weight-row byte offset per subtile
#pragma unroll
  for (int sb = 0; sb < NSUB; ++sb) bro[sb] = (sb * 32 + m) * 128;
  const int bsw = ((m >> 1) & 7);  // (r >> 1) & 7 for r = sb*32 + m
  f32x16 acc[NSUB], accx[NSUB];
#pragma unroll
  for (int sb = 0; sb < NSUB; ++sb) {
    acc[sb] = f32x16{};
    accx[sb] = f32x16{};
  }
  // read cursor of this wave's K-group: K-steps g, g+2, g+4, ...
  int c_t = 0, c_ky = 0, c_kx = 0, c_bs = 0, c_ps = 0;
  auto step_cursor = [&]() {
    ++c_kx;
    if (c_kx == KW) {
      c_kx = 0;
      ++c_ky;
    }
    c_bs = c_bs + 1 == SB ? 0 : c_bs + 1;
    if (++c_t == T) {
      c_t = 0;
      c_ky = 0;
      c_ps = c_ps + 1 == PA ? 0 : c_ps + 1;
    }
  };
  if (g == 1) step_cursor();
  struct Frag {
    f32x4 av[4];
    h8 bh[NSUB][2], bl[NSUB][2];
  };
  // the K-step under the read cursor: A (fp32) and weight (pre-split) fragments
  auto read_frag = [&](Frag& F) {
#ifdef HALO_ABL_NOREAD  // timing ablation (dev builds only): no fragment reads
    F.av[0] = f32x4{(float)c_ps, (float)c_bs, (float)c_ky, (float)c_kx};
    step_cursor();
    step_cursor();
    return;
#endif
    const char* Ab = smem + LDS_B + c_ps * (PI * 1024);
    const char* Bb = smem + c_bs * (BNT * 128);
    const int pp = ppbase + (c_ky * PW + c_kx);
    const int sw = (((m & 15) + c_kx) >> 1) & 7;  // swizzle of patch column px
#pragma unroll
    for (int jq = 0; jq < 4; ++jq)
      F.av[jq] = *reinterpret_cast<const f32x4*>(Ab + pp * 128 + (((4 * h + jq) ^ sw) << 4));
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        F.bh[sb][qq] = *reinterpret_cast<const h8*>(Bb + bro[sb] + (((2 * h + qq) ^ bsw) << 4));
        if constexpr (X3) F.bl[sb][qq] = *reinterpret_cast<const h8*>(Bb + bro[sb] + (((4 + 2 * h + qq) ^ bsw) << 4));
      }
    }
    step_cursor();
    step_cursor();
  };
  auto mfma_frag = [&](const Frag& F) {
    h8 ah[2], al[2];
#ifdef HALO_ABL_NOSPLIT  // timing ablation (dev builds only): bit casts instead of the split
    ah[0] = __builtin_bit_cast(h8, F.av[0]);
    al[0] = __builtin_bit_cast(h8, F.av[1]);
    ah[1] = __builtin_bit_cast(h8, F.av[2]);
    al[1] = __builtin_bit_cast(h8, F.av[3]);
#else
    split8<X3>(F.av[0], F.av[1], ah[0], al[0]);
    split8<X3>(F.av[2], F.av[3], ah[1], al[1]);
#endif
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb) {
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        acc[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], F.bh[sb][qq], acc[sb], 0, 0, 0);
        if constexpr (X3) {
          acc[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(al[qq], F.bh[sb][qq], acc[sb], 0, 0, 0);
          accx[sb] = __builtin_amdgcn_mfma_f32_32x32x16_f16(ah[qq], F.bl[sb][qq], accx[sb], 0, 0, 0);
        }
      }
    }
  };

  // ---- pipeline ------------------------------------------------------------
  // Super-step s: issue load set s+D; read the fragments of K-step 2(s+1)+g
  // (load set s+1) while the MFMAs of K-step 2s+g run on the registers read
  // last super-step; wait until load set s+2 has landed; one barrier.
  // hist[k] = this wave's DMA count of the load set issued k super-steps ago.
  constexpr int NH = D - 3 > 0 ? D - 3 : 1;
  int hist[NH];
  {
    int cnt[D];
#pragma unroll
    for (int u = 0; u < D; ++u) cnt[u] = issue_set();
    int n = 0;
#pragma unroll
    for (int u = 2; u < D; ++u) n += cnt[u];
    wait_vm_n(n);  // load sets 0 and 1 have landed
#pragma unroll
    for (int k = 0; k < NH; ++k) hist[k] = D - 1 - k >= 3 ? cnt[D - 1 - k] : 0;
  }
  __builtin_amdgcn_s_barrier();
  Frag F0, F1;
  if (g < nk) read_frag(F0);
#ifdef STAMPS
  unsigned long long t_iss = 0, t_cmp = 0, t_wait = 0, t_bar = 0, t0 = hstamp_now();
  const unsigned long long t_begin = t0;
#endif
  auto super_step = [&](int s, Frag& Fc, Frag& Fn) {
#ifdef STAMPS
    unsigned long long t1 = hstamp_now();
    t_iss += t1 - t0;
#endif
    const int nnew = issue_set();  // load set s + D
    if (2 * (s + 1) + g < nk) read_frag(Fn);
#ifdef HALO_ABL_NOMFMA  // timing ablation (dev builds only): fragments consumed, no MFMA
    if (2 * s + g < nk) acc[0][0] += Fc.av[0][0] + (float)Fc.bh[0][0][0];
#else
    if (2 * s + g < nk) mfma_frag(Fc);
#endif
#ifdef STAMPS
    unsigned long long t2 = hstamp_now();
    t_cmp += t2 - t1;
#endif
    // in flight after load set s+2: sets s+3 .. s+D
    int n = nnew;
#pragma unroll
    for (int k = 0; k < D - 3; ++k) n += hist[k];
#ifndef HALO_ABL_NOWAIT  // timing ablation (dev builds only): no DMA wait in the loop
    wait_vm_n(n);
#endif
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): the next fragments are in registers
#ifdef STAMPS
    unsigned long long t3 = hstamp_now();
    t_wait += t3 - t2;
#endif
#ifndef HALO_ABL_NOBAR  // timing ablation (dev builds only)
    __builtin_amdgcn_s_barrier();  // set s+2 readable by every wave; set s+1's reads done
#endif
#ifdef STAMPS
    t0 = hstamp_now();
    t_bar += t0 - t3;
#endif
#pragma unroll
    for (int k = NH - 1; k > 0; --k) hist[k] = hist[k - 1];
    hist[0] = nnew;
  };
  for (int s = 0; s < ns; s += 2) {
    super_step(s, F0, F1);
    if (s + 1 < ns) super_step(s + 1, F1, F0);
  }

#ifdef STAMPS
  {
    const unsigned wid = blockIdx.x * 8 + w;
    if (lane == 0 && wid < 16384) {
      g_hstamp[wid * 4 + 0] = t_iss;
      g_hstamp[wid * 4 + 1] = t_cmp;
      g_hstamp[wid * 4 + 2] = t_wait;
      g_hstamp[wid * 4 + 3] = t_bar;
    }
    (void)t_begin;
  }
#endif
  if constexpr (X3) {
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[sb][r] += accx[sb][r] * (1.0f / SPLIT_SCALE);
  }
  // K-group 1 hands its partial sums to group 0 through LDS (every DMA has landed)
  float* red = reinterpret_cast<float*>(smem);
  if (g == 1) {
#pragma unroll
    for (int sb = 0; sb < NSUB; ++sb)
#pragma unroll
      for (int r = 0; r < 16; ++r) red[((sb * 16 + r) * 4 + wm) * 64 + lane] = acc[sb][r];
  }
  __syncthreads();
  if (g == 1) return;
#pragma unroll
  for (int sb = 0; sb < NSUB; ++sb)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[sb][r] += red[((sb * 16 + r) * 4 + wm) * 64 + lane];

  // ---- epilogue: register r holds tile row m = (r&3) + 8(r>>2) + 4h of this wave's 32
  int rows[16];
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
    const int y = y0 + 2 * wm + (mm >> 4), x = x0 + (mm & 15);
    rows[r] = (y < p.out_h && x < p.out_w) ? (b * p.out_h + y) * p.out_w + x : -1;
  }
#pragma unroll
  for (int sb = 0; sb < NSUB; ++sb) tile_epilogue(p, rows, n0 + sb * 32 + m, acc[sb]);
}

template <int KH, int KW, int PREC>
void launch_halo_p(const HaloArgs& a, int bn, dim3 grid, hipStream_t s) {
  if (bn == 64)
    hipLaunchKernelGGL((conv_halo_kernel<KH, KW, 64, PREC>), grid, dim3(512), 0, s, a);
  else
    hipLaunchKernelGGL((conv_halo_kernel<KH, KW, 32, PREC>), grid, dim3(512), 0, s, a);
}
template <int KH, int KW>
void launch_halo_k(const HaloArgs& a, int bn, dim3 grid, hipStream_t s) {
  if (a.p.precision == RAFT_PREC_F16X3)
    launch_halo_p<KH, KW, RAFT_PREC_F16X3>(a, bn, grid, s);
  else
    launch_halo_p<KH, KW, RAFT_PREC_F16>(a, bn, grid, s);
}

}  // namespace

#ifdef STAMPS
extern "C" int raft_debug_hstamps(unsigned long long* host, int n) {
  return (int)hipMemcpyFromSymbol(host, HIP_SYMBOL(g_hstamp), sizeof(unsigned long long) * (size_t)n);
}
#endif

// Launches the halo kernel when the conv is one it covers (stride 1, "same"
// padding, 1x1 / 3x3 / 1x5 / 5x1, VEC mode, split-weight precisions);
// returns 1 without launching otherwise.  Arguments are already validated by
// raft_conv2d.
int conv_halo_launch(const raft_conv2d_params& p, int k_pad, int n_pad, unsigned w_bytes, unsigned in0_bytes,
                     unsigned in1_bytes, hipStream_t s) {
  static const bool enabled = [] {
    const char* e = getenv("RAFT_CONV_HALO");
    return !(e && e[0] == '0');
  }();
  if (!enabled) return 1;
  if (p.mode != RAFT_CONV_VEC || p.stride_h != 1 || p.stride_w != 1) return 1;
  if (p.precision != RAFT_PREC_F16X3 && p.precision != RAFT_PREC_F16) return 1;
  const int kh = p.kh, kw = p.kw;
  const bool shape = (kh == 1 && kw == 1) || (kh == 3 && kw == 3) || (kh == 1 && kw == 5) || (kh == 5 && kw == 1);
  if (!shape || p.pad_h != (kh - 1) / 2 || p.pad_w != (kw - 1) / 2) return 1;
  if (p.out_h != p.in_h || p.out_w != p.in_w || p.n <= 4) return 1;
  HaloArgs a;
  a.p = p;
  a.K = k_pad;
  a.nch = k_pad / (kh * kw) / 32;
  a.nk = a.nch * kh * kw;
  a.tx_n = cdiv(p.out_w, HTW);
  a.ty_n = cdiv(p.out_h, HTH);
  a.w_bytes = w_bytes;
  a.in0_bytes = in0_bytes;
  a.in1_bytes = in1_bytes;
  const long spatial = (long)p.batch * a.tx_n * a.ty_n;
  // one work-group per CU (LDS): 64 output channels per work-group unless
  // 32 still fits the grid in one round of 256 CUs with half of them idle at 64
  const int bn = spatial * (n_pad / 64) > 128 ? 64 : 32;
  a.gn = n_pad / bn;
  const long tiles = spatial * a.gn;
  if (tiles >= (1L << 31)) return 1;
  dim3 grid((unsigned)tiles);
  if (kh == 1 && kw == 1)
    launch_halo_k<1, 1>(a, bn, grid, s);
  else if (kh == 3)
    launch_halo_k<3, 3>(a, bn, grid, s);
  else if (kh == 1)
    launch_halo_k<1, 5>(a, bn, grid, s);
  else
    launch_halo_k<5, 1>(a, bn, grid, s);
  return 0;
}

}  // namespace raft
