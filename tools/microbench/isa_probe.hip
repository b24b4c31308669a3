// Probe: semantics + issue throughput of the SAD-family VALU ops on gfx950.
// Used to pick the cost-aggregation instruction mix.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>

typedef unsigned short us2 __attribute__((ext_vector_type(2)));

__global__ void sem(const uint32_t* in, uint64_t* out) {
  if (threadIdx.x != 0) return;
  uint32_t a = in[0], b = in[1], c = in[2], e = in[3];
  uint64_t s0 = ((uint64_t)b << 32) | a;
  uint64_t acc = ((uint64_t)0xFFF0u << 48) | ((uint64_t)3u << 32) | ((uint64_t)2u << 16) | 1u;
  out[0] = __builtin_amdgcn_qsad_pk_u16_u8(s0, c, acc);
  out[1] = __builtin_amdgcn_mqsad_pk_u16_u8(s0, c, acc);
  out[2] = __builtin_amdgcn_sad_u8(a, c, 7);
  out[3] = __builtin_amdgcn_sad_hi_u8(a, c, 7);
  out[4] = __builtin_amdgcn_msad_u8(a, c, 7);
  out[5] = __builtin_amdgcn_msad_u8(c, a, 7);
  out[6] = __builtin_amdgcn_mqsad_pk_u16_u8(s0, e, 0);
  out[7] = __builtin_amdgcn_sad_u16(a, c, 0);
}

template <int OP>
__global__ void thr(const uint32_t* in, uint32_t* out, int iters) {
  uint32_t x = in[threadIdx.x & 7], y = in[(threadIdx.x + 3) & 7];
  uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
  uint64_t q0 = a0, q1 = a1, q2 = a2, q3 = a3, q4 = a4, q5 = a5, q6 = a6, q7 = a7;
  uint64_t s0 = ((uint64_t)y << 32) | x;
  for (int i = 0; i < iters; ++i) {
#define STEP(A) \
    if constexpr (OP == 0) A = __builtin_amdgcn_sad_u8(x, y, A); \
    if constexpr (OP == 1) A = __builtin_amdgcn_sad_hi_u8(x, y, A); \
    if constexpr (OP == 2) A = __builtin_amdgcn_msad_u8(x, y, A); \
    if constexpr (OP == 5) { us2 t = __builtin_bit_cast(us2, A); t = t + __builtin_bit_cast(us2, x); A = __builtin_bit_cast(uint32_t, t); } \
    if constexpr (OP == 6) A = __builtin_amdgcn_perm(A, x, 0x0C050400u); \
    if constexpr (OP == 7) A = __builtin_amdgcn_alignbyte(A, x, y & 3); \
    if constexpr (OP == 8) A = min(min(A, x), y) ; \
    if constexpr (OP == 9) A = A + x;
#define QSTEP(Q) \
    if constexpr (OP == 3) Q = __builtin_amdgcn_qsad_pk_u16_u8(s0, y, Q); \
    if constexpr (OP == 4) Q = __builtin_amdgcn_mqsad_pk_u16_u8(s0, y, Q);
    STEP(a0) STEP(a1) STEP(a2) STEP(a3) STEP(a4) STEP(a5) STEP(a6) STEP(a7)
    QSTEP(q0) QSTEP(q1) QSTEP(q2) QSTEP(q3) QSTEP(q4) QSTEP(q5) QSTEP(q6) QSTEP(q7)
    x ^= i;  // defeat hoisting
  }
  out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 +
      (uint32_t)(q0 + q1 + q2 + q3 + q4 + q5 + q6 + q7);
}

template <int OP>
void run(const char* name, const uint32_t* din, uint32_t* dout) {
  const int blocks = 256 * 8, threads = 256, iters = 4096;
  hipEvent_t e0, e1; hipEventCreate(&e0); hipEventCreate(&e1);
  thr<OP><<<blocks, threads>>>(din, dout, iters);
  hipDeviceSynchronize();
  hipEventRecord(e0);
  for (int r = 0; r < 5; ++r) thr<OP><<<blocks, threads>>>(din, dout, iters);
  hipEventRecord(e1); hipEventSynchronize(e1);
  float ms; hipEventElapsedTime(&ms, e0, e1); ms /= 5;
  double wave_instr = (double)blocks * (threads / 64) * iters * 8.0;
  // per CU per ns -> per clock at 2.4 GHz is only nominal (DVFS)
  double per_cu_per_us = wave_instr / 256.0 / (ms * 1e3);
  printf("%-22s %8.3f ms  %8.1f wave-instr/CU/us  (= %.2f per CU-clk @2.4GHz; 2.0 = full-rate VALU)\n",
         name, ms, per_cu_per_us, per_cu_per_us / 2400.0);
}

int main() {
  uint32_t h[8] = {0x00FF1005u, 0x40302010u, 0x05000A03u, 0xFF000000u, 1, 2, 3, 4};
  uint32_t *din, *dout; uint64_t* dsem;
  hipMalloc(&din, 64); hipMalloc(&dout, 256 * 8 * 256 * 4); hipMalloc(&dsem, 64);
  hipMemcpy(din, h, 32, hipMemcpyHostToDevice);
  sem<<<1, 64>>>(din, dsem);
  uint64_t r[8]; hipMemcpy(r, dsem, 64, hipMemcpyDeviceToHost);
  printf("a=%08x b=%08x c=%08x e=%08x acc=fff0.0003.0002.0001\n", h[0], h[1], h[2], h[3]);
  const char* nm[8] = {"qsad_pk(s0,c,acc)", "mqsad_pk(s0,c,acc)", "sad_u8(a,c,7)", "sad_hi_u8(a,c,7)",
                       "msad_u8(a,c,7)", "msad_u8(c,a,7)", "mqsad_pk(s0,e,0)", "sad_u16(a,c,0)"};
  for (int i = 0; i < 8; ++i) printf("  %-20s = %016llx\n", nm[i], (unsigned long long)r[i]);
  run<0>("v_sad_u8", din, dout);
  run<1>("v_sad_hi_u8", din, dout);
  run<2>("v_msad_u8", din, dout);
  run<3>("v_qsad_pk_u16_u8", din, dout);
  run<4>("v_mqsad_pk_u16_u8", din, dout);
  run<5>("v_pk_add_u16", din, dout);
  run<6>("v_perm_b32", din, dout);
  run<7>("v_alignbyte_b32", din, dout);
  run<8>("v_min3_u32", din, dout);
  run<9>("v_add_u32", din, dout);
  return 0;
}
