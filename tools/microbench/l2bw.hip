// Microbenchmark: L2 -> CU read bandwidth with register loads (global_load_dwordx4), one
// workgroup per CU, every workgroup sweeping the same L2-resident buffer (the pattern of
// the chain's weight stream).  Prints GB/s per CU for waves-per-workgroup x loads in flight.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int DEPTH>
__global__ void sweep(const u32x4* __restrict__ buf, int n16, int reps, unsigned* sink) {
  const int nw = blockDim.x >> 6, w = threadIdx.x >> 6, lane = threadIdx.x & 63;
  u32x4 acc = {0, 0, 0, 0};
  u32x4 r[DEPTH];
  // wave w reads 1 KiB chunks w, w + nw, ... (64 lanes x 16 B), DEPTH chunks per round
  const int chunks = n16 / 64;
  int c = w;
  for (int rep = 0; rep < reps; ++rep) {
    for (int base = 0; base < chunks; base += nw * DEPTH) {
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) {
        int cc = base + w + d * nw;
        cc = cc < chunks ? cc : cc - chunks;
        r[d] = buf[cc * 64 + lane];
      }
#pragma unroll
      for (int d = 0; d < DEPTH; ++d) acc ^= r[d];
    }
  }
  (void)c;
  if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) sink[0] = 1;
}

template <int DEPTH>
void run(const u32x4* buf, int n16, unsigned* sink, int waves, int cus) {
  const int reps = 20;
  hipEvent_t a, b;
  (void)hipEventCreate(&a);
  (void)hipEventCreate(&b);
  sweep<DEPTH><<<cus, waves * 64>>>(buf, n16, 2, sink);
  (void)hipEventRecord(a);
  sweep<DEPTH><<<cus, waves * 64>>>(buf, n16, reps, sink);
  (void)hipEventRecord(b);
  (void)hipEventSynchronize(b);
  float ms = 0;
  (void)hipEventElapsedTime(&ms, a, b);
  const double bytes = (double)n16 * 16 * reps;  // per workgroup
  printf("waves %d depth %2d cus %3d: %.1f GB/s per CU, %.2f TB/s chip\n", waves, DEPTH, cus, bytes / (ms * 1e-3) / 1e9,
         bytes * cus / (ms * 1e-3) / 1e12);
}

int main() {
  const int n16 = 256 * 1024 / 16;  // 256 KiB buffer
  u32x4* buf;
  unsigned* sink;
  (void)hipMalloc(&buf, n16 * 16);
  (void)hipMalloc(&sink, 4);
  (void)hipMemset(buf, 1, n16 * 16);
  for (int cus : {256, 32}) {
    for (int waves : {4, 8, 16}) {
      run<4>(buf, n16, sink, waves, cus);
      run<8>(buf, n16, sink, waves, cus);
      run<16>(buf, n16, sink, waves, cus);
      run<32>(buf, n16, sink, waves, cus);
    }
  }
  return 0;
}
