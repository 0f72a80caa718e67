// Shared pieces of the conv GEMM kernels (conv_gemm.hip, conv_halo.hip):
// operand types, the fp32 split, buffer descriptors and the fused epilogues.
#pragma once

#include "common.hpp"

namespace raft {
namespace {

using h4 = __attribute__((ext_vector_type(4))) _Float16;
using v4u = __attribute__((ext_vector_type(4))) unsigned;
using h8 = __attribute__((ext_vector_type(8))) _Float16;
using bf4 = __attribute__((ext_vector_type(4))) __bf16;
using bf8 = __attribute__((ext_vector_type(8))) __bf16;

// bf16 operands travel in the f16 containers (same 16-bit lanes): round to
// nearest even (v_cvt_pk_bf16_f32), bit-cast at the MFMA
__device__ __forceinline__ h4 to_bf16x4(const f32x4 x) {
  return __builtin_bit_cast(h4, __builtin_convertvector(x, bf4));
}

constexpr float SPLIT_SCALE = 2048.f;  // lo is stored scaled by 2^11 (kept out of f16 subnormals)

// x = hi + lo / 2048 to ~22 bits: hi = f16(x); x - hi is exact in fp32, its
// 2^11-scaled value rounds to f16 lo.
__device__ __forceinline__ void split4(const f32x4 x, h4& hi, h4& lo) {
#pragma unroll
  for (int e = 0; e < 4; ++e) {
    const _Float16 h = (_Float16)x[e];
    hi[e] = h;
    lo[e] = (_Float16)((x[e] - (float)h) * SPLIT_SCALE);
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

// 8 floats -> 8 f16 hi (+ 8 f16 lo = f16(x - hi)) : 4 VALU per 2 elements;
// BF: 8 bf16 (round to nearest even) in the f16 container, no lo
template <bool LO, bool BF = false>
__device__ __forceinline__ void split8(const f32x4 x0, const f32x4 x1, h8& hi, h8& lo) {
  if constexpr (BF) {
    const h4 a = to_bf16x4(x0), b = to_bf16x4(x1);
    hi = h8{a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
    return;
  }
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

__device__ __forceinline__ float sigmoidf_(float v) { return 1.0f / (1.0f + expf(-v)); }

__device__ __forceinline__ void epilogue(const raft_conv2d_params& p, long m, int n, float v) {
  if (p.add0) v += p.add0[m * p.add0_ld + n];
  float* o = p.out + m * p.out_ld + n;
  switch (p.epilogue) {
    case RAFT_EPI_LINEAR:
      *o = p.alpha * v;
      break;
    case RAFT_EPI_RELU:
      *o = fmaxf(v, 0.f);
      break;
    case RAFT_EPI_RESID_RELU:
      *o = fmaxf(p.aux0[m * p.aux0_ld + n] + fmaxf(v, 0.f), 0.f);
      break;
    case RAFT_EPI_GRU_ZR:
      if (n < p.split) {
        *o = sigmoidf_(v);
      } else {
        const int c = n - p.split;
        p.out1[m * p.out1_ld + c] = sigmoidf_(v) * p.aux0[m * p.aux0_ld + c];
      }
      break;
    case RAFT_EPI_GRU_Q: {
      const float q = tanhf(v);
      const float z = p.aux1[m * p.aux1_ld + n];
      const float h = p.aux0[m * p.aux0_ld + n];
      *o = (1.0f - z) * h + z * q;
      break;
    }
    case RAFT_EPI_TANH_RELU:
      if (n < p.split)
        *o = tanhf(v);
      else
        p.out1[m * p.out1_ld + (n - p.split)] = fmaxf(v, 0.f);
      break;
    case RAFT_EPI_ADD_TO_OUT:
      *o = *o + v;
      break;
    default:
      break;
  }
}

// Epilogue of one 32x32 MFMA tile: lane owns column n and the 16 rows
// mb + (r&3) + 8*(r>>2).  All operand loads of the 16 rows (add0, aux0/aux1,
// the ADD_TO_OUT destination) are issued together from clamped addresses
// before any store, and only the stores are predicated: on gfx9 stores share
// vmcnt with loads, so a row-by-row load/store interleave would wait for every
// earlier store to complete (one full write latency per row).
__device__ __forceinline__ long row_of(int mb, int r) { return mb + (r & 3) + 8 * (r >> 2); }

// rows[r] = the output pixel (GEMM row) of accumulator register r, or -1 past
// the edge (its loads read row 0, its store is dropped).  Element indices are
// 32-bit (rows * ld < 2^30, host-checked), so each address is one VGPR offset
// from the scalar base.
__device__ __forceinline__ unsigned eidx(int row, int ld, int col) {
  return (unsigned)(row < 0 ? 0 : row) * (unsigned)ld + (unsigned)col;
}
// WT: sc1 loads (served past the CU's L1: data another work-group of the launch wrote through)
template <bool WT = false, int R0 = 0, int RN = 16>
__device__ __forceinline__ void load_rows(const float* base, int ld, const int (&rows)[16], int col, float (&t)[16]) {
#pragma unroll
  for (int r = R0; r < R0 + RN; ++r) {
    if constexpr (WT)
      t[r] = __hip_atomic_load(base + eidx(rows[r], ld, col), __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else
      t[r] = base[eidx(rows[r], ld, col)];
  }
}

// branch-free activations (no per-row control flow between the stores)
__device__ __forceinline__ float sigmoid_bf(float x) { return __frcp_rn(1.0f + __expf(-x)); }
__device__ __forceinline__ float tanh_bf(float x) { return 1.0f - 2.0f * __frcp_rn(__expf(2.0f * x) + 1.0f); }

constexpr int CPOL_SC1 = 16;  // buffer cache-policy bit sc1 (gfx950): write-through to memory
constexpr unsigned OFF_INVALID = 0x80000000u;  // > num_records of every buffer (host-checked)

// 4x4 transpose across the four lanes of a quad: lane q's x[i] <- lane i's x[q] (two exchange
// steps, with lane q^1 then lane q^2, by DPP quad permutes)
__device__ __forceinline__ void quad_transpose(float (&x)[4]) {
  const int q = threadIdx.x & 3;
  float y[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float nb = __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, x[i ^ 1]), 0xB1, 0xF, 0xF, false));
    y[i] = ((i ^ q) & 1) ? nb : x[i];
  }
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    const float nb = __builtin_bit_cast(
        float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, y[i ^ 2]), 0x4E, 0xF, 0xF, false));
    x[i] = ((i ^ q) & 2) ? nb : y[i];
  }
}

// Stores one 32x32 MFMA tile's values (lane: column col, rows[r] of register r, -1 = none) as
// 16-B buffer stores: a quad transpose gives each lane 4 consecutive columns of one row, rows past
// the edge get an out-of-range offset (dropped by the buffer's range check), so there is no
// per-element branch and no 64-bit address math.  nq = the conv column of the lane's quad start,
// ncols = the conv's N (a quad straddling it stores its valid columns one by one).  Needs a 16-B
// aligned dst and ld % 4 == 0 (the caller checks).  CPOL: the buffer cache policy (CPOL_SC1 =
// write-through).
template <int CPOL>
__device__ __forceinline__ void store_tile16(float* dst, int ld, long nrows, const int (&rows)[16], int col, int nq,
                                             int ncols, const float (&v)[16]) {
  const int q = threadIdx.x & 3;
  const unsigned c0 = (unsigned)(col - q);
  const long bytes = nrows * (long)ld * 4;
  const __amdgpu_buffer_rsrc_t rs =
      __builtin_amdgcn_make_buffer_rsrc(dst, (short)0, (int)(bytes < 0x7FFFFFF0L ? bytes : 0x7FFFFFF0L), 0x00020000);
  const bool full = nq + 3 < ncols, part = !full && nq < ncols;
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    float x[4] = {v[4 * j], v[4 * j + 1], v[4 * j + 2], v[4 * j + 3]};
    quad_transpose(x);
    const int row = q == 0 ? rows[4 * j] : q == 1 ? rows[4 * j + 1] : q == 2 ? rows[4 * j + 2] : rows[4 * j + 3];
    const unsigned off = row >= 0 ? ((unsigned)row * (unsigned)ld + c0) * 4u : OFF_INVALID;
    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(v4u, f32x4{x[0], x[1], x[2], x[3]}), rs,
                                           full ? off : OFF_INVALID, 0, CPOL);
    if (part) {
#pragma unroll
      for (int i = 0; i < 4; ++i)
        if (nq + i < ncols) __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(unsigned, x[i]), rs, off + 4u * i, 0, CPOL);
    }
  }
}

// WT: write-through stores (sc1: the bytes leave the XCD's L2 at once)
// R0, RN: only accumulator rows R0 .. R0 + RN - 1 (the K-split form's halves, halo_body KS = 2)
template <bool WT = false, int R0 = 0, int RN = 16>
__device__ __forceinline__ void tile_epilogue(const raft_conv2d_params& p, const int (&rows)[16], int n,
                                              const f32x16& acc) {
  static_assert(!WT || (R0 == 0 && RN == 16), "write-through epilogues store whole 16-row tiles");
  const bool ncol = n < p.n;
  const int nc = ncol ? n : p.n - 1;  // clamped column for loads
  float v[16];
  const float bias = p.bias ? p.bias[nc] : 0.f;
#pragma unroll
  for (int r = R0; r < R0 + RN; ++r) v[r] = acc[r] + bias;
  if (p.add0) {
    float t[16];
    load_rows<WT, R0, RN>(p.add0, p.add0_ld, rows, nc, t);
#pragma unroll
    for (int r = R0; r < R0 + RN; ++r) v[r] += t[r];
  }
  // 1) operand loads, 2) values, 3) stores: destination dst[row * ld + col]
  float* dst = p.out;
  int ld = p.out_ld, col = n;
  const int epi = p.epilogue;
  if (epi == RAFT_EPI_LINEAR) {
#pragma unroll
    for (int r = R0; r < R0 + RN; ++r) v[r] *= p.alpha;
  } else if (epi == RAFT_EPI_RELU) {
#pragma unroll
    for (int r = R0; r < R0 + RN; ++r) v[r] = fmaxf(v[r], 0.f);
  } else if (epi == RAFT_EPI_RESID_RELU) {
    float t[16];
    load_rows<WT, R0, RN>(p.aux0, p.aux0_ld, rows, nc, t);
#pragma unroll
    for (int r = R0; r < R0 + RN; ++r) v[r] = fmaxf(t[r] + fmaxf(v[r], 0.f), 0.f);
  } else if (epi == RAFT_EPI_GRU_ZR) {
    if (nc < p.split) {  // a wave's 32 columns lie on one side of split (split % 32 == 0, host-checked)
#pragma unroll
      for (int r = R0; r < R0 + RN; ++r) v[r] = sigmoid_bf(v[r]);
    } else {
      col = nc - p.split;
      float t[16];
      load_rows<WT, R0, RN>(p.aux0, p.aux0_ld, rows, col, t);
#pragma unroll
      for (int r = R0; r < R0 + RN; ++r) v[r] = sigmoid_bf(v[r]) * t[r];
      dst = p.out1;
      ld = p.out1_ld;
    }
  } else if (epi == RAFT_EPI_GRU_Q) {
    float h[16], z[16];
    load_rows<WT, R0, RN>(p.aux0, p.aux0_ld, rows, nc, h);
    load_rows<WT, R0, RN>(p.aux1, p.aux1_ld, rows, nc, z);
#pragma unroll
    for (int r = R0; r < R0 + RN; ++r) v[r] = (1.0f - z[r]) * h[r] + z[r] * tanh_bf(v[r]);
  } else if (epi == RAFT_EPI_TANH_RELU) {
    if (nc < p.split) {
#pragma unroll
      for (int r = R0; r < R0 + RN; ++r) v[r] = tanh_bf(v[r]);
    } else {
#pragma unroll
      for (int r = R0; r < R0 + RN; ++r) v[r] = fmaxf(v[r], 0.f);
      dst = p.out1;
      ld = p.out1_ld;
      col = n - p.split;
    }
  } else if (epi == RAFT_EPI_ADD_TO_OUT) {
    float t[16];
    load_rows<WT, R0, RN>(p.out, p.out_ld, rows, nc, t);
#pragma unroll
    for (int r = R0; r < R0 + RN; ++r) v[r] += t[r];
  }
  if (p.range_flag) {  // f16x3 range guard (raft_hip.h): out-of-range outputs raise the flag
    bool big = false;
#pragma unroll
    for (int r = R0; r < R0 + RN; ++r) big |= ncol && rows[r] >= 0 && fabsf(v[r]) > RAFT_RANGE_LIMIT;
    if (big) *p.range_flag = 1;
  }
  // write-through outputs: 16-B stores (a 4-B sc1 store is a fabric write of its own); plain
  // outputs keep the per-element stores (the 16-B form measured 3.7 % slower on the update convs)
  if (WT && (((uintptr_t)dst) & 15) == 0 && (ld & 3) == 0) {
    store_tile16<WT ? CPOL_SC1 : 0>(dst, ld, (long)p.batch * p.out_h * p.out_w, rows, col, n - (threadIdx.x & 3), p.n, v);
    return;
  }
#pragma unroll
  for (int r = R0; r < R0 + RN; ++r)
    if (ncol && rows[r] >= 0) {
      if constexpr (WT)
        __hip_atomic_store(dst + eidx(rows[r], ld, col), v[r], __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      else
        dst[eidx(rows[r], ld, col)] = v[r];
    }
}

// InstanceNorm partial statistics of one wave's 32x32 accumulator tile (raft_conv2d_stats_slots):
// for column n, (count, mean, M2) of v = acc + bias over the wave's valid rows; lanes n and n + 32
// hold 16 rows each.  M2 is taken around the wave's own mean (well conditioned in fp32).
// (count, mean, M2) of one 32-pixel block's rows of column n (every lane of the wave gets them)
__device__ __forceinline__ f32x4 tile_stats_vals(const int (&rows)[16], const f32x16& acc, float bias) {
  float s = 0.f, c = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    s += rows[r] >= 0 ? acc[r] + bias : 0.f;
    c += rows[r] >= 0 ? 1.f : 0.f;
  }
  s += __shfl_xor(s, 32);
  c += __shfl_xor(c, 32);
  const float mean = c > 0.f ? s / c : 0.f;
  float m2 = 0.f;
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const float d = acc[r] + bias - mean;
    m2 += rows[r] >= 0 ? d * d : 0.f;
  }
  m2 += __shfl_xor(m2, 32);
  return f32x4{c, mean, m2, 0.f};
}
// Chan's combination of two (count, mean, M2) partials
__device__ __forceinline__ f32x4 stats_combine(const f32x4& a, const f32x4& b) {
  const float n = a[0] + b[0];
  if (b[0] <= 0.f) return a;
  if (a[0] <= 0.f) return b;
  const float d = b[1] - a[1];
  return f32x4{n, a[1] + d * (b[0] / n), a[2] + b[2] + d * d * (a[0] * b[0] / n), 0.f};
}
__device__ __forceinline__ void stats_write(const raft_conv2d_params& p, int n, long slot, const f32x4& v) {
  if (n < p.n && (threadIdx.x & 32) == 0)
    *reinterpret_cast<f32x4*>(p.stats_part + (slot * p.stats_ld + n) * 4) = v;
}
__device__ __forceinline__ void tile_stats_b(const raft_conv2d_params& p, const int (&rows)[16], int n,
                                             const f32x16& acc, long slot, float bias) {
  stats_write(p, n, slot, tile_stats_vals(rows, acc, bias));
}
__device__ __forceinline__ void tile_stats(const raft_conv2d_params& p, const int (&rows)[16], int n,
                                           const f32x16& acc, long slot) {
  tile_stats_b(p, rows, n, acc, slot, p.bias ? p.bias[n < p.n ? n : 0] : 0.f);
}


__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int CPOL = 0>
__device__ __forceinline__ f32x4 buf_load4(__amdgpu_buffer_rsrc_t r, unsigned voff, unsigned soff) {
  return __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, voff, soff, CPOL));
}

// LDS-DMA of 16 B per lane (buffer_load ... lds: 1 KiB per wave instruction)
__device__ __forceinline__ void dma16(__amdgpu_buffer_rsrc_t rs, void* lds, unsigned voff, unsigned soff) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)lds, 16, voff, soff, 0, 0);
}

// s_waitcnt vmcnt(n) only (expcnt / lgkmcnt at their maxima)
template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | 0x70 | 0xF00 | ((N >> 4) << 14));
}
// n > 15 waits for 15 (stricter than needed, never looser)
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

}  // namespace

// a validated conv with its packed-weight shape and operand byte sizes (raft_conv2d)
struct HaloOperands {
  raft_conv2d_params p;
  int k_pad, n_pad;
  unsigned w_bytes, in0_bytes, in1_bytes;
};

// conv_halo.hip: the halo-tiled LDS-DMA kernel for stride-1 "same" convs;
// returns 1 (nothing launched) when the conv is not one it covers
int conv_halo_launch(const HaloOperands& o, hipStream_t s);
// two independent convs of one shape class in one launch; 1 (nothing launched) if they do not qualify
int conv_halo_launch_pair(const HaloOperands& o0, const HaloOperands& o1, hipStream_t s);
// conv_stem.hip: the encoders' 7x7 / stride-2 stem over 3 channels; 1 (nothing launched) otherwise
int conv_stem_launch(const raft_conv2d_params& p, int k_pad, hipStream_t s);
// tile-statistics slots per image of a conv on the halo / stem kernel (raft_conv2d_stats_slots), 0 if none
int conv_halo_stats_slots(const HaloOperands& o);
// whether conv_halo_launch takes the conv
bool conv_halo_covers(const HaloOperands& o);
int conv_halo_tile_rows(const HaloOperands& o);
int conv_halo_tiles_per_wg(const HaloOperands& o);
bool conv_halo_norm_ok(const HaloOperands& o);
int conv_stem_stats_slots(const raft_conv2d_params& p, int k_pad);

}  // namespace raft
