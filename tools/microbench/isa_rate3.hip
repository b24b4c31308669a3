// Issue rates of candidate VOP3 ops (chains use lane-varying operands so nothing folds).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

template <int OP> __device__ __forceinline__ uint32_t op(uint32_t a, uint32_t x, uint32_t y) {
  if constexpr (OP == 0) return (a << 8) | x;                                  // v_lshl_or_b32
  if constexpr (OP == 1) return __builtin_amdgcn_ubfe(a ^ x, 8, 16);          // v_bfe_u32 (+xor)
  if constexpr (OP == 2) return min(min(a, x), y);                           // v_min3_u32
  if constexpr (OP == 3) return a + x + y;                                     // v_add3_u32
  if constexpr (OP == 4) return (a & 0xFFFFu) * 256u + x;                      // mad_u32_u16 / lshl_or?
  if constexpr (OP == 5) return a ^ x;                                         // v_xor_b32
  if constexpr (OP == 6) return (uint32_t)__builtin_amdgcn_sbfe((int)(a ^ x), 3, 1);  // v_bfe_i32
  if constexpr (OP == 7) { uint64_t s0 = ((uint64_t)y << 32) | a; return (uint32_t)__builtin_amdgcn_mqsad_pk_u16_u8(s0, x, (uint64_t)a); }
  if constexpr (OP == 8) return __builtin_amdgcn_sad_u8(a, x, y);
  if constexpr (OP == 9) return min(a, x);
  if constexpr (OP == 10) return (a & x) | y;
  if constexpr (OP == 11) return __builtin_amdgcn_perm(a, x, y);
  if constexpr (OP == 12) return a & x;
  if constexpr (OP == 13) return a >> (x & 7);
  if constexpr (OP == 14) return a + x;
  if constexpr (OP == 15) return a - x;
  if constexpr (OP == 16) return a | x;
  if constexpr (OP == 17) return (a >> 8) ^ x;
  if constexpr (OP == 18) { float f = __builtin_bit_cast(float, a); float g = __builtin_bit_cast(float, x); return __builtin_bit_cast(uint32_t, __builtin_fmaf(f, g, 1.0f)); }
  if constexpr (OP == 19) return __builtin_amdgcn_sad_hi_u8(a, x, y);
  return a;
}

template <int OP>
__global__ void thr(const uint32_t* in, uint32_t* out, int iters) {
  uint32_t xs[8], y = in[(threadIdx.x + 3) & 7] | 0x0C0C0000u;
#pragma unroll
  for (int c = 0; c < 8; ++c) xs[c] = in[(threadIdx.x + c) & 7] + c;
  uint32_t acc[8];
#pragma unroll
  for (int c = 0; c < 8; ++c) acc[c] = threadIdx.x * 7 + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int c = 0; c < 8; ++c) acc[c] = op<OP>(acc[c], xs[(c + k) & 7], y);
#pragma unroll
      for (int c = 0; c < 8; ++c) asm volatile("" : "+v"(acc[c]));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < 8; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP> void report(const char* name, const uint32_t* din, uint32_t* dout) {
  const int blocks = 256 * 8, iters = 1024;
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  thr<OP><<<blocks, 256>>>(din, dout, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) thr<OP><<<blocks, 256>>>(din, dout, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  // per SIMD: 8 waves x iters*64 instr
  double cyc = ms * 1e-3 * 2.4e9 / (8.0 * iters * 64);
  printf("%-26s SIMD cycles per wave-instr: %5.2f\n", name, cyc);
}

int main() {
  uint32_t h[8] = {0x00FF1005u, 0x40302010u, 0x05000A03u, 0x0C0C0504u, 1, 2, 3, 4};
  uint32_t *din, *dout;
  (void)hipMalloc(&din, 64); (void)hipMalloc(&dout, 256 * 8 * 256 * 4);
  (void)hipMemcpy(din, h, 32, hipMemcpyHostToDevice);
  report<18>("v_fma_f32 (ref)", din, dout);
  report<14>("v_add_u32", din, dout);
  report<15>("v_sub_u32", din, dout);
  report<12>("v_and_b32", din, dout);
  report<16>("v_or_b32", din, dout);
  report<5>("v_xor_b32", din, dout);
  report<13>("v_lshrrev(+and)", din, dout);
  report<17>("lshr8^x", din, dout);
  report<9>("v_min_u32", din, dout);
  report<2>("v_min3_u32", din, dout);
  report<10>("v_and_or_b32", din, dout);
  report<8>("v_sad_u8", din, dout);
  report<19>("v_sad_hi_u8", din, dout);
  report<11>("v_perm_b32", din, dout);
  return 0;
}
