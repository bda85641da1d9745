// Microbenchmark: L2 -> CU read bandwidth of a continuous register ring (the chain3 /
// lgemm weight stream): each wave keeps DEPTH 1 KiB loads in flight, consuming the oldest
// before issuing the next; every workgroup (one per CU x WPC) sweeps the same L2-resident
// buffer, each wave its own slice.
#include <hip/hip_runtime.h>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int DEPTH>
__global__ void ring(const u32x4* __restrict__ buf, int chunks_per_wave, int reps, unsigned* sink) {
  const int nw = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4* base = buf + (size_t)w * chunks_per_wave * 64 + lane;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[DEPTH];
  const int total = chunks_per_wave * reps;
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) r[d] = base[(d % chunks_per_wave) * 64];
  for (int i0 = 0; i0 < total; i0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc ^= r[d];
      const int nxt = (i0 + d + DEPTH) % chunks_per_wave;
      r[d] = base[nxt * 64];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) acc ^= r[d];
  (void)nw;
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

// the same sweep with the last `dma_waves` waves of each workgroup streaming through
// direct-to-LDS loads (global_load_lds_dwordx4 into a per-wave 8 KiB LDS ring, vmcnt-paced)
typedef __attribute__((address_space(3))) void lds_void;
template <int DEPTH>
__global__ void ring_dma(const u32x4* __restrict__ buf, int chunks_per_wave, int reps, unsigned* sink, int dma_waves) {
  __shared__ __attribute__((aligned(16))) char lds[16 * 8 * 1024];
  const int nw = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const u32x4* base = buf + (size_t)w * chunks_per_wave * 64 + lane;
  const int total = chunks_per_wave * reps;
  if (w >= nw - dma_waves) {
    char* ring = lds + w * 8 * 1024;
    for (int i = 0; i < total; ++i) {
      __builtin_amdgcn_global_load_lds(base + (i % chunks_per_wave) * 64, (lds_void*)(ring + (i & 7) * 1024), 16, 0, 0);
      asm volatile("s_waitcnt vmcnt(7)" ::: "memory");
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    if (ring[lane] == 123) sink[1] = 1;
    return;
  }
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[DEPTH];
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) r[d] = base[(d % chunks_per_wave) * 64];
  for (int i0 = 0; i0 < total; i0 += DEPTH) {
#pragma unroll
    for (int d = 0; d < DEPTH; ++d) {
      acc ^= r[d];
      const int nxt = (i0 + d + DEPTH) % chunks_per_wave;
      r[d] = base[nxt * 64];
      __builtin_amdgcn_sched_barrier(0);
    }
  }
#pragma unroll
  for (int d = 0; d < DEPTH; ++d) acc ^= r[d];
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <int DEPTH>
void run_dma(const u32x4* buf, unsigned* sink, int waves, int dma_waves) {
  const int chunks_per_wave = 32, reps = 64, grid = 256;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  ring_dma<DEPTH><<<grid, waves * 64>>>(buf, chunks_per_wave, 4, sink, dma_waves);
  (void)hipEventRecord(a);
  ring_dma<DEPTH><<<grid, waves * 64>>>(buf, chunks_per_wave, reps, sink, dma_waves);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double bytes_cu = (double)waves * chunks_per_wave * 1024 * reps;
  printf("waves/WG %2d (%d of them LDS-DMA) depth %2d: %.1f GB/s per CU\n", waves, dma_waves, DEPTH, bytes_cu / (ms * 1e-3) / 1e9);
}

template <int DEPTH>
void run(const u32x4* buf, unsigned* sink, int waves, int wgs_per_cu) {
  const int chunks_per_wave = 32;  // 32 KiB per wave (a chain phase)
  const int reps = 64;
  const int grid = 256 * wgs_per_cu;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  ring<DEPTH><<<grid, waves * 64>>>(buf, chunks_per_wave, 4, sink);
  (void)hipEventRecord(a);
  ring<DEPTH><<<grid, waves * 64>>>(buf, chunks_per_wave, reps, sink);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double bytes_cu = (double)waves * wgs_per_cu * chunks_per_wave * 1024 * reps;
  printf("waves/WG %2d WG/CU %d depth %2d: %.1f GB/s per CU\n", waves, wgs_per_cu, DEPTH, bytes_cu / (ms * 1e-3) / 1e9);
}

int main() {
  u32x4* buf;
  unsigned* sink;
  (void)hipMalloc(&buf, 16 * 32 * 1024);  // 16 waves x 32 KiB
  (void)hipMalloc(&sink, 4);
  (void)hipMemset(buf, 1, 16 * 32 * 1024);
  for (int waves : {4, 8, 12, 16}) {
    for (int wpc : {1}) {
      run<8>(buf, sink, waves, wpc);
      run<16>(buf, sink, waves, wpc);
      run<32>(buf, sink, waves, wpc);
    }
  }
  for (int dw : {0, 1, 2, 4}) {
    run_dma<8>(buf, sink, 8 + dw, dw);
    run_dma<16>(buf, sink, 8 + dw, dw);
  }
  return 0;
}
