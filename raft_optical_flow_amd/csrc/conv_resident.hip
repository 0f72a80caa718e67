// Weight-resident persistent 3x3 convolution for the feature / context encoders' stride-1 convs
// over <= 96 input channels (core/extractor.py:6-56, ResidualBlock conv1 / conv2 of layer1 and
// layer2), gfx950.
//
// Why: at 1/2 resolution these convs are 1792 (config 2) to 8000 (1080x1920) output tiles of the
// halo kernel with only 18 K-steps each (K = 64 x 9), so a one-tile work-group spends most of its
// life in its prologue (first weights + patch from L2) and epilogue; the grid runs 7+ rounds of
// that.  Here a work-group owns ONE 32-column N-tile for the whole launch: its split weights
// (K x 32 x (hi | lo) = 72 KB for 64 channels, 108 KB for 96) are loaded into LDS once, and it
// walks its spatial tiles as one continuous stream of 32-channel patch chunks: the loader waves
// keep the patches of the next two chunks in flight (registers) and one pre-split chunk ahead in
// LDS while the MFMA waves run the current one, so a tile's epilogue overlaps the next tile's
// patch loads and no weight byte is re-read per tile.
//
// Work-group: 4 MFMA waves (wave w: tile rows 2w, 2w+1 = 32 pixels x 32 columns, one 32x32 MFMA
// block, f16x3: hi*hi + lo*hi + hi*(2048 lo) as in conv_halo.hip) + 4 loader waves, one per CU;
// grid = 8 x gn x m work-groups (gn N-tiles), so the gn work-groups sharing a spatial sequence
// are g, g + 8, ... (one XCD under round-robin dispatch: their patches meet in one L2).
// One s_barrier per chunk (9 K-steps).  Epilogues, InstanceNorm partials (stats_part) and the
// input InstanceNorm (in_norm, the per-image table held in LDS) as the halo kernel's.
#include "conv_common.hpp"

namespace raft {
namespace {

constexpr int RTW = 16, RTH = 8;                                  // output tile (pixels)
constexpr int RPW = RTW + 2, RPH = RTH + 2, RNPIX = RPH * RPW;    // 3x3 patch: 10 x 18
constexpr int RPI = (RNPIX + 7) / 8;                              // 1-KiB pieces per patch slot
constexpr int RBN = 32;                                           // columns per work-group
constexpr int RWROW = 128;                                        // split weight row (hi | lo) per K-step
constexpr int RES_LDS = 160 * 1024;
constexpr int RES_PATCH = 2 * RPI * 1024;                         // two patch slots
constexpr int RNB = 4;                                            // patch chunks in flight per loader lane

struct ResArgs {
  raft_conv2d_params p;
  int K;                   // packed weight row length (floats)
  int nch;                 // 32-channel chunks (<= 3)
  int gn;                  // N-tiles (32 columns each) that hold real columns
  int tx_n, ty_n, spatial; // spatial tiles per image / in all images
  int groups;              // work-groups per N-tile
  unsigned w_bytes, in0_bytes;
  int patch_off, tab_off;  // LDS byte offsets: patch slots, input-norm table
};

template <bool NORM, int EPI>
__global__ __launch_bounds__(512) void conv_resident_kernel(const ResArgs ra) {
  __shared__ __attribute__((aligned(1024))) char smem[RES_LDS];
  const raft_conv2d_params& p = ra.p;
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const bool loader = w >= 4;
  const int lw = w & 3;
  // work-group -> (N-tile nt, spatial sequence grp, grp + groups, ...)
  const int xcd = blockIdx.x & 7, slot = blockIdx.x >> 3;
  const int nt = slot % ra.gn;
  const int grp = xcd + 8 * (slot / ra.gn);
  const int nch = ra.nch, nk = 9 * nch;
  const int ntile = grp < ra.spatial ? (ra.spatial - 1 - grp) / ra.groups + 1 : 0;
  const int NI = ntile * nch;  // chunk steps (uniform per work-group)
  if (NI == 0) return;
  const int per = ra.tx_n * ra.ty_n;
  auto tile_of = [&](int k, int& st, int& b, int& y0, int& x0) {
    st = grp + k * ra.groups;
    b = st / per;
    const int sr = st - b * per;
    y0 = (sr / ra.tx_n) * RTH;
    x0 = (sr % ra.tx_n) * RTW;
  };

  // ---- the work-group's split weights: packed K-step jj (tap t, chunk c: jj = t * nch + c) of
  // rows nt*32 .. +31 -> LDS block jj (32 rows x 128 B, 16-B quads XOR-swizzled by (row >> 1) & 7)
  {
    const __amdgpu_buffer_rsrc_t rs_w = make_rsrc(p.weight, ra.w_bytes);
    for (int pc = w; pc < nk * 4; pc += 8) {
      const int jj = pc >> 2, r = (pc & 3) * 8 + (lane >> 3);
      const int qd = (lane & 7) ^ ((r >> 1) & 7);
      dma16(rs_w, smem + jj * (RBN * RWROW) + (pc & 3) * 1024,
            (unsigned)(nt * RBN + r) * ((unsigned)ra.K * 4u) + (unsigned)qd * 16u, (unsigned)jj * 128u);
    }
  }
  float* norm_tab = reinterpret_cast<float*>(smem + ra.tab_off);
  if constexpr (NORM) {  // {mean, rstd} of every (image, input channel)
    const int n = 2 * p.batch * p.in0_c;
    for (int i = threadIdx.x; i < n; i += 512) norm_tab[i] = p.in_norm[i];
  }

  if (loader) {
    // ---- loader waves: 8-channel patch tasks t = (patch pixel t / 4, channel group t % 4) ----
    const __amdgpu_buffer_rsrc_t rs0 = make_rsrc(p.in0, ra.in0_bytes);
    const int in0_c = p.in0_c, in_h = p.in_h, in_w = p.in_w;
    const unsigned ld0 = p.in0_ld;
    constexpr int NT = 4 * RNPIX, TI = (NT + 255) / 256;
    int tpy[TI], tpx[TI], tlds[TI], tg8[TI];
#pragma unroll
    for (int i = 0; i < TI; ++i) {
      const int t = 64 * lw + lane + 256 * i;
      const int pp = t >> 2, gq = t & 3;
      tpy[i] = pp / RPW;
      tpx[i] = pp - tpy[i] * RPW;
      tg8[i] = 8 * gq;
      tlds[i] = t < NT ? pp * 128 + ((gq ^ ((tpx[i] >> 1) & 7)) << 4) : -1;
    }
    using Staged = f32x4[TI][2];
    auto pix_ok = [&](int i, int y0, int x0, int& pix, int b) {
      const int iy = y0 + tpy[i] - 1, ix = x0 + tpx[i] - 1;
      pix = (b * in_h + iy) * in_w + ix;
      return tlds[i] >= 0 && (unsigned)iy < (unsigned)in_h && (unsigned)ix < (unsigned)in_w;
    };
    auto load_chunk = [&](int ci, Staged& dst) {
      const int k = ci / nch, c = ci - k * nch;
      int st, b, y0, x0;
      tile_of(k, st, b, y0, x0);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        int pix;
        const bool ok = pix_ok(i, y0, x0, pix, b);
#pragma unroll
        for (int q = 0; q < 2; ++q) {
          const int ch = 32 * c + tg8[i] + 4 * q;
          const unsigned voff = ok && ch < in0_c ? ((unsigned)pix * ld0 + (unsigned)ch) * 4u : OFF_INVALID;
          dst[i][q] = buf_load4(rs0, voff, 0);
        }
      }
    };
    auto store_chunk = [&](int ci, const Staged& src) {
      const int k = ci / nch, c = ci - k * nch;
      int st, b, y0, x0;
      tile_of(k, st, b, y0, x0);
      char* base = smem + ra.patch_off + (ci & 1) * (RPI * 1024);
#pragma unroll
      for (int i = 0; i < TI; ++i) {
        if (tlds[i] < 0) continue;
        h8 hi, lo;
        if constexpr (NORM) {
          int pix;
          const bool ok = pix_ok(i, y0, x0, pix, b);
          const int ch = 32 * c + tg8[i];
          float e[8] = {src[i][0][0], src[i][0][1], src[i][0][2], src[i][0][3],
                        src[i][1][0], src[i][1][1], src[i][1][2], src[i][1][3]};
#pragma unroll
          for (int j = 0; j < 8; ++j) {
            const bool okj = ok && ch + j < in0_c;
            const float2 mr = reinterpret_cast<const float2*>(norm_tab)[okj ? b * in0_c + ch + j : 0];
            const float v = (e[j] - mr.x) * mr.y;
            e[j] = okj ? (p.in_norm_relu ? fmaxf(v, 0.f) : v) : 0.f;
          }
          split8<true, false>(f32x4{e[0], e[1], e[2], e[3]}, f32x4{e[4], e[5], e[6], e[7]}, hi, lo);
        } else {
          split8<true, false>(src[i][0], src[i][1], hi, lo);
        }
        *reinterpret_cast<h8*>(base + tlds[i]) = hi;
        *reinterpret_cast<h8*>(base + (tlds[i] ^ 64)) = lo;
      }
    };
    // RNB register sets of patch loads in flight (the loads are latency-bound: MALL-served input,
    // one 23-KB chunk per set).  Chunk ci lives in set ci % RNB.
    // prologue: chunk 0 stored (slot 0); chunks 1 .. RNB in flight
    Staged pv[RNB];
    load_chunk(0, pv[0]);
    wait_vm<0>();     // (the weights too)
    __syncthreads();  // the norm table (all waves) is in LDS
    store_chunk(0, pv[0]);
#pragma unroll
    for (int j = 1; j <= RNB; ++j)
      if (j < NI) load_chunk(j, pv[j % RNB]);
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0)
    __builtin_amdgcn_s_barrier();        // B0
    // step i: store chunk i+1 (its loads are the oldest in flight) into slot (i+1) & 1 (it held
    // chunk i-1, read during step i-1), then issue chunk i+1+RNB into the freed register set
    auto step = [&](int i, Staged& set) {
      if (i + 1 < NI) {
        const int newer = (NI - 1 - (i + 1)) < RNB - 1 ? NI - 1 - (i + 1) : RNB - 1;  // chunks issued after i+1
        switch (newer) {
          case 0: wait_vm<0>(); break;
          case 1: wait_vm<2 * TI>(); break;
          case 2: wait_vm<4 * TI>(); break;
          default: wait_vm<(RNB - 1) * 2 * TI>(); break;
        }
#ifndef RES_ABL_NOLOAD  // timing ablations (dev builds only)
        store_chunk(i + 1, set);
        if (i + 1 + RNB < NI) load_chunk(i + 1 + RNB, set);
#endif
      }
      __builtin_amdgcn_s_waitcnt(0xC07F);
      __builtin_amdgcn_s_barrier();  // B(i+1): chunk i+1 readable, slot i free
    };
    for (int i = 0; i < NI; i += RNB) {
#pragma unroll
      for (int j = 0; j < RNB; ++j)
        if (i + j < NI) step(i + j, pv[(j + 1) % RNB]);
    }
    wait_vm<0>();
    return;
  }

  // ---- MFMA waves ------------------------------------------------------------------------
  const int m = lane & 31, h = lane >> 5;
  const int bsw = (m >> 1) & 7;
  const int ppb = (2 * w + (m >> 4)) * RPW + (m & 15);  // patch pixel of this lane's row (tap 0, 0)
  f32x16 acc = f32x16{}, accx = f32x16{};
  // the lane's output column is fixed for the launch: its bias once, not per tile
  const int ncol = nt * RBN + m;
  const bool colok = ncol < p.n;
  const float bias = p.bias ? p.bias[colok ? ncol : p.n - 1] : 0.f;
  constexpr bool resid = EPI == RAFT_EPI_RESID_RELU;
  // the epilogue's operands, hoisted out of the tile loop
  float* const out = p.out;
  const int out_ld = p.out_ld;
  const long nrows = (long)p.batch * p.out_h * p.out_w;
  const float alpha = p.alpha;
  int* const range_flag = p.range_flag;
  float aux[16];  // the residual rows of the tile being finished (loaded before its last chunk)
  auto tile_rows = [&](int k, int (&rows)[16], int& st) {
    int b, y0, x0;
    tile_of(k, st, b, y0, x0);
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int mm = (r & 3) + 8 * (r >> 2) + 4 * h;
      const int y = y0 + 2 * w + (mm >> 4), x = x0 + (mm & 15);
      rows[r] = (y < p.out_h && x < p.out_w) ? (b * p.out_h + y) * p.out_w + x : -1;
    }
  };
  struct Frag {
    h8 ah[2], al[2], bh[2], bl[2];
  };
  wait_vm<0>();     // this wave's weight DMAs
  __syncthreads();  // the norm table
  __builtin_amdgcn_s_barrier();  // B0: weights, chunk 0
  for (int i = 0; i < NI; ++i) {
    const int k = i / nch, c = i - k * nch;
    const char* Ab = smem + ra.patch_off + (i & 1) * (RPI * 1024);
    auto read = [&](Frag& F, int t) {
      const int ky = t / 3, kx = t - 3 * ky;
      const char* Bb = smem + (t * nch + c) * (RBN * RWROW) + m * RWROW;
      const char* row = Ab + (ppb + ky * RPW + kx) * 128;
      const int sw = (((m & 15) + kx) >> 1) & 7;
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        F.bh[qq] = *reinterpret_cast<const h8*>(Bb + (((2 * h + qq) ^ bsw) << 4));
        F.bl[qq] = *reinterpret_cast<const h8*>(Bb + (((4 + 2 * h + qq) ^ bsw) << 4));
        F.ah[qq] = *reinterpret_cast<const h8*>(row + (((2 * h + qq) ^ sw) << 4));
        F.al[qq] = *reinterpret_cast<const h8*>(row + (((4 + 2 * h + qq) ^ sw) << 4));
      }
    };
    if (resid && c == nch - 1) {  // the epilogue's operand loads fly under the last chunk's MFMAs
      int rows[16], st;
      tile_rows(k, rows, st);
      load_rows(p.aux0, p.aux0_ld, rows, colok ? ncol : p.n - 1, aux);
    }
    Frag F[2];
    read(F[0], 0);
#pragma unroll
    for (int t = 0; t < 9; ++t) {
      if (t + 1 < 9) read(F[(t + 1) & 1], t + 1);
#ifndef RES_NOPIN  // keep the next tap's reads ahead of this tap's MFMAs (the scheduler sinks them otherwise)
      __builtin_amdgcn_sched_barrier(0);
#endif
      const Frag& G = F[t & 1];
#ifdef RES_ABL_NOMFMA
      asm volatile("" ::"v"(G.ah[0]), "v"(G.bh[0]), "v"(G.al[1]), "v"(G.bl[1]), "v"(G.ah[1]), "v"(G.bh[1]), "v"(G.al[0]), "v"(G.bl[0]));
#else
#pragma unroll
      for (int qq = 0; qq < 2; ++qq) {
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(G.ah[qq], G.bh[qq], acc, 0, 0, 0);
        accx = __builtin_amdgcn_mfma_f32_32x32x16_f16(G.ah[qq], G.bl[qq], accx, 0, 0, 0);
        acc = __builtin_amdgcn_mfma_f32_32x32x16_f16(G.al[qq], G.bh[qq], acc, 0, 0, 0);
      }
#endif
#ifndef RES_NOPIN
      __builtin_amdgcn_sched_barrier(0);
#endif
    }
#ifdef RES_ABL_NOEPI
    if (c == nch - 1 && acc[0] == 12345.f) {
#else
    if (c == nch - 1) {
#endif
      // the tile's epilogue (the loaders meanwhile stream the next tile's first chunks)
#pragma unroll
      for (int r = 0; r < 16; ++r) acc[r] += accx[r] * (1.0f / SPLIT_SCALE);
      int rows[16], st;
      tile_rows(k, rows, st);
      if (p.stats_part) tile_stats_b(p, rows, ncol, acc, (long)st * 4 + w, bias);
      // LINEAR / RELU / RESID_RELU (conv_resident_launch admits no other), branch-free
      float v[16];
      bool big = false;
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const float t = acc[r] + bias;
        v[r] = resid ? fmaxf(aux[r] + fmaxf(t, 0.f), 0.f) : (EPI == RAFT_EPI_RELU ? fmaxf(t, 0.f) : alpha * t);
        big |= colok && rows[r] >= 0 && fabsf(v[r]) > RAFT_RANGE_LIMIT;
      }
      if (range_flag && big) *range_flag = 1;
#ifdef RES_ABL_NOSTORE
      asm volatile("" ::"v"(v[0]), "v"(v[5]), "v"(v[10]), "v"(v[15]), "v"(rows[3]), "v"(rows[12]));
#else
#pragma unroll
      for (int r = 0; r < 16; ++r)
        if (colok && rows[r] >= 0) out[eidx(rows[r], out_ld, ncol)] = v[r];
#endif
      acc = f32x16{};
      accx = f32x16{};
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0): this chunk's fragment reads are done
    __builtin_amdgcn_s_barrier();        // B(i+1)
  }
}

int res_grid_limit() {
  static const int cus = [] {
    int dev = 0, n = 0;
    if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess)
      return 0;
    return n;
  }();
  return cus;
}

// opt-in (RAFT_RESIDENT=1; read per call: tests switch it): on the same box it measured no faster
// than the one-tile halo kernel
bool resident_enabled() {
  const char* e = getenv("RAFT_RESIDENT");
  return e && e[0] == '1';
}

}  // namespace

// The weight-resident kernel's view of a conv it covers: 3x3 stride 1 "same", one input segment of
// <= 96 channels, f16x3, and a grid of more than two rounds of one-tile work-groups; 1 (nothing
// launched) otherwise.
int conv_resident_launch(const HaloOperands& o, hipStream_t s) {
  const raft_conv2d_params& p = o.p;
  if (!resident_enabled()) return 1;
  if (p.mode != RAFT_CONV_VEC || p.precision != RAFT_PREC_F16X3 || p.kh != 3 || p.kw != 3 || p.stride_h != 1 ||
      p.stride_w != 1 || p.pad_h != 1 || p.pad_w != 1 || p.out_h != p.in_h || p.out_w != p.in_w || p.in1_c != 0 ||
      p.n <= 4)
    return 1;
  ResArgs ra;
  ra.p = p;
  ra.K = o.k_pad;
  ra.nch = o.k_pad / 9 / 32;
  if (ra.nch < 1 || ra.nch > 3 || ra.nch * 32 < p.in0_c) return 1;
  ra.gn = cdiv(p.n, RBN);
  ra.tx_n = cdiv(p.out_w, RTW);
  ra.ty_n = cdiv(p.out_h, RTH);
  const long spatial = (long)p.batch * ra.tx_n * ra.ty_n;
  if (p.add0 || (p.epilogue != RAFT_EPI_LINEAR && p.epilogue != RAFT_EPI_RELU && p.epilogue != RAFT_EPI_RESID_RELU))
    return 1;
  const int cus = res_grid_limit();
  if (cus < 8 * ra.gn || spatial * ra.gn <= 2L * cus || spatial >= (1L << 30)) return 1;
  ra.spatial = (int)spatial;
  const int mult = cus / (8 * ra.gn);
  ra.groups = 8 * mult;
  ra.w_bytes = o.w_bytes;
  ra.in0_bytes = o.in0_bytes;
  ra.patch_off = 9 * ra.nch * RBN * RWROW;
  ra.tab_off = ra.patch_off + RES_PATCH;
  const long tab = p.in_norm ? 8L * p.batch * p.in0_c : 0;
  if (ra.tab_off + tab > RES_LDS) return 1;
  // (store_tile16: 16-B aligned output rows)
  if ((((uintptr_t)p.out) & 15) != 0 || (p.out_ld & 3) != 0) return 1;
  const dim3 grid((unsigned)(ra.groups * ra.gn));
  const bool nrm = p.in_norm != nullptr;
  switch (p.epilogue) {
    case RAFT_EPI_LINEAR:
      if (nrm) hipLaunchKernelGGL((conv_resident_kernel<true, RAFT_EPI_LINEAR>), grid, dim3(512), 0, s, ra);
      else hipLaunchKernelGGL((conv_resident_kernel<false, RAFT_EPI_LINEAR>), grid, dim3(512), 0, s, ra);
      break;
    case RAFT_EPI_RELU:
      if (nrm) hipLaunchKernelGGL((conv_resident_kernel<true, RAFT_EPI_RELU>), grid, dim3(512), 0, s, ra);
      else hipLaunchKernelGGL((conv_resident_kernel<false, RAFT_EPI_RELU>), grid, dim3(512), 0, s, ra);
      break;
    default:
      if (nrm) hipLaunchKernelGGL((conv_resident_kernel<true, RAFT_EPI_RESID_RELU>), grid, dim3(512), 0, s, ra);
      else hipLaunchKernelGGL((conv_resident_kernel<false, RAFT_EPI_RESID_RELU>), grid, dim3(512), 0, s, ra);
      break;
  }
  return 0;
}

}  // namespace raft
