// Per-CU L2 -> LDS ingest-rate microbenchmark (dev tool, not part of the library).
//
// One 512-thread work-group per CU streams 1-KiB pieces (8 rows x 128 B, the
// conv kernels' piece shape) from an L2-resident table into an LDS ring:
//   mode 0: LDS-DMA (buffer_load_dwordx4 ... lds), counted vmcnt, raw barrier;
//   mode 1: register staging (buffer_load_dwordx4 -> ds_write_b128), the same
//           pieces and ring.
// Build: hipcc -O3 --offload-arch=gfx950 tools/ingest_bench.hip -o tools/ingest_bench
// Run:   tools/ingest_bench <mode> <loader_waves> <pieces_per_wave_per_step> <steps_in_flight>
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <type_traits>
#include <utility>

using f32x4 = __attribute__((ext_vector_type(4))) float;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t make_rsrc(const void* p, unsigned bytes) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(p), (short)0, (int)bytes, 0x00020000);
}

template <int N>
__device__ __forceinline__ void wait_vm() {
  __builtin_amdgcn_s_waitcnt((N & 15) | 0x70 | 0xF00 | ((N >> 4) << 14));
}

// STEPS super-steps; per super-step each loader wave moves PPW pieces; ring of
// (DEPTH+1) slots of (LW*PPW) KiB.  Row r of piece: table row ((blk*7919 + r*131) % rows).
template <int MODE, int LW, int PPW, int DEPTH>
__global__ __launch_bounds__(512, 1) void ingest(const float* table, unsigned rows, int steps, float* sink) {
#if defined(__HIP_DEVICE_COMPILE__)
  constexpr int SLOT = LW * PPW * 1024;
  constexpr int NS = DEPTH + 1;
  static_assert(NS * SLOT <= 160 * 1024, "LDS");
  __shared__ __attribute__((aligned(1024))) char lds[NS * SLOT];
  const int lane = threadIdx.x & 63;
  const int w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  const auto rs = make_rsrc(table, rows * 128u);
  float acc = 0.f;
  auto voff_of = [&](int s, int k) {
    const unsigned blk = (unsigned)((blockIdx.x * 977 + s * 61 + (w * PPW + k) * 13) % (rows / 8));
    return (blk * 8u + (unsigned)(lane >> 3)) * 128u + (unsigned)(lane & 7) * 16u;
  };
  f32x4 reg[DEPTH + 1][PPW];
  auto issue = [&](int s, auto slot_c) {
    constexpr int slot = decltype(slot_c)::value;
    if (w >= LW) return;
#pragma unroll
    for (int k = 0; k < PPW; ++k) {
      if constexpr (MODE == 0) {
        __builtin_amdgcn_raw_ptr_buffer_load_lds(rs, (__attribute__((address_space(3))) void*)(lds + slot * SLOT + (w * PPW + k) * 1024), 16,
                                                 voff_of(s, k), 0, 0, 0);
      } else {
        reg[slot][k] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(rs, voff_of(s, k), 0, 0));
      }
    }
  };
  auto step = [&](int s, auto slot_c) {
    constexpr int slot = decltype(slot_c)::value;
    issue(s + DEPTH, std::integral_constant<int, (slot + DEPTH) % NS>{});
    if constexpr (MODE == 0) {
      if (w < LW) wait_vm<(DEPTH) * PPW>();
    } else {
      if (w < LW) {
        wait_vm<(DEPTH) * PPW>();
#pragma unroll
        for (int k = 0; k < PPW; ++k)
          *reinterpret_cast<f32x4*>(lds + slot * SLOT + (w * PPW + k) * 1024 + lane * 16) = reg[slot][k];
      }
    }
    __builtin_amdgcn_s_waitcnt(0xC07F);
    __builtin_amdgcn_s_barrier();
    acc += *reinterpret_cast<const float*>(lds + slot * SLOT + (threadIdx.x * 4) % SLOT);
  };
  [&]<int... U>(std::integer_sequence<int, U...>) { (issue(U, std::integral_constant<int, U>{}), ...); }(
      std::make_integer_sequence<int, DEPTH>{});
  for (int s = 0; s + NS <= steps; s += NS) {
    [&]<int... U>(std::integer_sequence<int, U...>) { (step(s + U, std::integral_constant<int, U>{}), ...); }(
        std::make_integer_sequence<int, NS>{});
  }
  if (acc == 1234.5f) sink[threadIdx.x] = acc;
#endif
}

#define CHECK(x)                                                             \
  do {                                                                       \
    hipError_t e = (x);                                                      \
    if (e != hipSuccess) {                                                   \
      fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e)); \
      exit(1);                                                               \
    }                                                                        \
  } while (0)

template <int MODE, int LW, int PPW, int DEPTH>
void run(const float* table, unsigned rows, float* sink, int cus) {
  const int steps = 420;  // a multiple of every ring size used
  hipEvent_t e0, e1;
  CHECK(hipEventCreate(&e0));
  CHECK(hipEventCreate(&e1));
  ingest<MODE, LW, PPW, DEPTH><<<cus, 512>>>(table, rows, steps, sink);
  CHECK(hipDeviceSynchronize());
  CHECK(hipEventRecord(e0));
  for (int r = 0; r < 5; ++r) ingest<MODE, LW, PPW, DEPTH><<<cus, 512>>>(table, rows, steps, sink);
  CHECK(hipEventRecord(e1));
  CHECK(hipEventSynchronize(e1));
  float ms;
  CHECK(hipEventElapsedTime(&ms, e0, e1));
  const double bytes = (double)steps * LW * PPW * 1024;  // per CU per launch
  const double s = ms / 5 * 1e-3;
  printf("mode %d (%s) loaders %d pieces/wave/step %d depth %d: %.2f us/launch, %.1f GB/s per CU, %.2f KiB in flight/CU\n",
         MODE, MODE ? "reg-staged" : "LDS-DMA", LW, PPW, DEPTH, s * 1e6, bytes / s / 1e9, (double)LW * PPW * DEPTH);
}

int main() {
  const unsigned rows = 16384;  // 2 MiB table: L2-resident after the first pass
  float *table, *sink;
  CHECK(hipMalloc(&table, rows * 128));
  CHECK(hipMalloc(&sink, 4096));
  CHECK(hipMemset(table, 0, rows * 128));
  const int cus = 256;
  run<0, 8, 1, 2>(table, rows, sink, cus);
  run<0, 8, 1, 4>(table, rows, sink, cus);
  run<0, 8, 2, 4>(table, rows, sink, cus);
  run<0, 8, 2, 6>(table, rows, sink, cus);
  run<0, 4, 2, 4>(table, rows, sink, cus);
  run<0, 4, 4, 4>(table, rows, sink, cus);
  run<0, 2, 4, 4>(table, rows, sink, cus);
  run<0, 8, 3, 4>(table, rows, sink, cus);
  run<1, 8, 1, 2>(table, rows, sink, cus);
  run<1, 8, 1, 4>(table, rows, sink, cus);
  run<1, 8, 2, 4>(table, rows, sink, cus);
  run<1, 8, 2, 6>(table, rows, sink, cus);
  run<1, 4, 4, 4>(table, rows, sink, cus);
  run<1, 8, 3, 4>(table, rows, sink, cus);
  return 0;
}
