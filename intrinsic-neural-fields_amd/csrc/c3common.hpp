// Device helpers shared by the register-streamed chains (chain3.hip: training step;
// rchain.hip: forward-only render / inference): LDS tile layouts, bf16 bit casts, DPP and
// permlane cross-lane sums, the LDS hand-off barrier.
#pragma once

#include <utility>

#include "common.hpp"

namespace inf {
namespace c3 {

typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));
typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));
typedef short s16x4x8 __attribute__((ext_vector_type(8)));

// byte offset of element (row, col) of a bf16 LDS tile with `rowb`-byte rows: 16-byte
// chunk c of row r stored at chunk c ^ (r & 15) (a ds_read_b128 lane group of 16 rows
// at one chunk is conflict-free)
__device__ __forceinline__ int tile_off(int rowb, int row, int col) {
  return row * rowb + (((col >> 3) ^ (row & 15)) << 4) + ((col & 7) << 1);
}

// The activation tile: per 32-feature k block q one 1 KiB block of B-operand fragments,
// slot (ray, g) = the 16 bytes of lane ray + 16 g, element e = feature 32 q + 16 (e / 4) +
// 4 g + e % 4 (accumulator order).  The slot of (ray, g) sits at ray ^ act_swz(q, g): the
// store wave's transposing reads (one ray of 16 row groups x 2 halves per 32-lane half)
// then hit 32 distinct 8-byte bank pairs, and the MFMA operand reads stay conflict-free
// (act_swz(q, g) ^ act_swz(q, g ^ 1) = 12 keeps the two row groups of every ds_read_b128
// lane group on complementary ray sets).
__device__ __forceinline__ int act_swz(int q, int g) { return ((q & 3) << 1) ^ ((g & 1) * 12) ^ (g >> 1); }
__device__ __forceinline__ int act_off(int q, int ray, int g) { return q * 1024 + (((ray ^ act_swz(q, g)) + 16 * g) << 4); }

__device__ __forceinline__ unsigned short bf_bits3(float x) {
  bf16 h = (bf16)x;
  return __builtin_bit_cast(unsigned short, h);
}
__device__ __forceinline__ float bf_val3(unsigned short u) { return (float)__builtin_bit_cast(bf16, u); }

template <int CTRL>
__device__ __forceinline__ float dpp_mov(float v) {
  return __builtin_bit_cast(float, __builtin_amdgcn_update_dpp(0, __builtin_bit_cast(int, v), CTRL, 0xF, 0xF, false));
}
constexpr int DPP_QUAD_1032 = 0xB1, DPP_QUAD_2301 = 0x4E, DPP_HALF_MIRROR = 0x141, DPP_MIRROR = 0x140,
              DPP_ROR4 = 0x124, DPP_ROR8 = 0x128;

// Sum over the 16 lanes of a row (lanes 16 q .. 16 q + 15) with DPP adds.
__device__ __forceinline__ float row_sum16(float v) {
  v += dpp_mov<DPP_QUAD_1032>(v);
  v += dpp_mov<DPP_QUAD_2301>(v);
  v += dpp_mov<DPP_HALF_MIRROR>(v);
  v += dpp_mov<DPP_MIRROR>(v);
  return v;
}

// One reduce-scatter step over a DPP lane pairing: v[0, 2M) -> v[0, M), keeping the half
// selected by `hi` and adding the partner lane's copy of it (the partner keeps the other).
template <int M, int CTRL>
__device__ __forceinline__ void halve(float* v, bool hi) {
#pragma unroll
  for (int i = 0; i < M; ++i) {
    const float keep = hi ? v[i + M] : v[i];
    const float give = hi ? v[i] : v[i + M];
    v[i] = keep + dpp_mov<CTRL>(give);
  }
}

// Sums over the 16 rays of a row group (lanes of a row) of NV values per lane, scattered:
// lane i returns the sum of value i % NV.  log2(NV) halving steps on pairings that flip
// lane bits {3} (NV = 16 only), {0,1,2}, {1}, {0} -- each keeps the lanes that still share
// a value set together -- then rotations complete the sum over the remaining lanes.
template <int NV>
__device__ __forceinline__ float ray_sum(float* v, int lane) {
  static_assert(NV == 4 || NV == 8 || NV == 16, "values per lane");
  if constexpr (NV == 16) halve<8, DPP_ROR8>(v, lane & 8);
  if constexpr (NV >= 8) halve<4, DPP_HALF_MIRROR>(v, lane & 4);
  halve<2, DPP_QUAD_2301>(v, lane & 2);
  halve<1, DPP_QUAD_1032>(v, lane & 1);
  if constexpr (NV == 4) v[0] += dpp_mov<DPP_ROR4>(v[0]);
  if constexpr (NV <= 8) v[0] += dpp_mov<DPP_ROR8>(v[0]);
  return v[0];
}

// Sum over lanes l, l ^ 16, l ^ 32, l ^ 48 (the four row groups of an accumulator column)
// with the gfx950 permlane swaps.  v_permlane16_swap x, y exchanges the odd 16-lane rows
// of x with the even rows of y: on two copies of v, x becomes v with odd rows <- even rows
// and y v with even rows <- odd rows, so x + y is the partner sum in every lane (32: the
// same with halves).  Inline asm: the ROCm 7.2 builtin returned the first register twice.
__device__ __forceinline__ float col_sum4(float v) {
  float x = v, y = v;
  asm volatile("s_nop 1\n\tv_permlane16_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  v = x + y;
  x = v;
  y = v;
  asm volatile("s_nop 1\n\tv_permlane32_swap_b32 %0, %1" : "+v"(x), "+v"(y));
  return x + y;
}

// ReLU as one v_max_f32 (fmaxf adds a canonicalising max per element; NaN -> 0 either way)
__device__ __forceinline__ float relu1(float x) {
  float r;
  asm("v_max_f32 %0, 0, %1" : "=v"(r) : "v"(x));
  return r;
}

// two floats -> packed bf16 pair (RNE, one v_cvt_pk_bf16_f32), a in the low half
typedef float f32x2_t __attribute__((ext_vector_type(2)));
typedef __bf16 bf16x2_t __attribute__((ext_vector_type(2)));
__device__ __forceinline__ unsigned pack_bf16x2(float a, float b) {
  return __builtin_bit_cast(unsigned, __builtin_convertvector(f32x2_t{a, b}, bf16x2_t));
}

// f(integral_constant<int, I>) for I = 0 .. N-1: a loop whose index is a compile-time
// constant in the body (ring slots statically indexed, per-step schedules unrolled)
template <typename F, int... I>
__device__ __forceinline__ void sfor_impl(F& f, std::integer_sequence<int, I...>) {
  (f(std::integral_constant<int, I>{}), ...);
}
template <int N, typename F>
__device__ __forceinline__ void sfor(F&& f) {
  sfor_impl(f, std::make_integer_sequence<int, N>{});
}

// LDS hand-off barrier that does not drain the vector-memory queue (__syncthreads()
// would add `s_waitcnt vmcnt(0)` and stall on the weight fragments in flight)
__device__ __forceinline__ void lbar() { asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory"); }


}  // namespace c3
}  // namespace inf
