// Issue-rate and dependent-latency probe for the VALU ops the matcher uses (gfx950).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
typedef unsigned short us2 __attribute__((ext_vector_type(2)));

template <int OP> __device__ __forceinline__ uint32_t op(uint32_t a, uint32_t x, uint32_t y) {
  if constexpr (OP == 0) return __builtin_amdgcn_sad_u8(x, y, a);
  if constexpr (OP == 1) return __builtin_amdgcn_sad_hi_u8(x, y, a);
  if constexpr (OP == 2) return __builtin_amdgcn_perm(a, x, y);
  if constexpr (OP == 3) return min(min(a, x), y);
  if constexpr (OP == 4) return a + x;
  if constexpr (OP == 5) return a - x;
  if constexpr (OP == 6) { us2 t = __builtin_bit_cast(us2, a) + __builtin_bit_cast(us2, x); return __builtin_bit_cast(uint32_t, t); }
  if constexpr (OP == 7) return __builtin_amdgcn_alignbyte(a, x, y);
  if constexpr (OP == 8) return (a & x) | y;
  if constexpr (OP == 9) return __builtin_amdgcn_msad_u8(x, y, a);
  if constexpr (OP == 10) return min(a, x);
  return a;
}

template <int OP, int CH>
__global__ void thr(const uint32_t* in, uint32_t* out, int iters) {
  uint32_t x = in[threadIdx.x & 7], y = in[(threadIdx.x + 3) & 7];
  uint32_t acc[CH];
#pragma unroll
  for (int c = 0; c < CH; ++c) acc[c] = threadIdx.x + c;
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
#pragma unroll
      for (int c = 0; c < CH; ++c) acc[c] = op<OP>(acc[c], x, y);
      asm volatile("" : "+v"(x));
    }
  }
  uint32_t s = 0;
#pragma unroll
  for (int c = 0; c < CH; ++c) s += acc[c];
  out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <int OP, int CH>
double run(int blocks, int iters, const uint32_t* din, uint32_t* dout) {
  hipEvent_t e0, e1; (void)hipEventCreate(&e0); (void)hipEventCreate(&e1);
  thr<OP, CH><<<blocks, 256>>>(din, dout, iters);
  (void)hipDeviceSynchronize();
  (void)hipEventRecord(e0);
  for (int r = 0; r < 3; ++r) thr<OP, CH><<<blocks, 256>>>(din, dout, iters);
  (void)hipEventRecord(e1); (void)hipEventSynchronize(e1);
  float ms; (void)hipEventElapsedTime(&ms, e0, e1); ms /= 3;
  double instr_per_wave = (double)iters * 8 * CH;
  return ms * 1e-3 * 2.4e9 / instr_per_wave;  // cycles per instruction per wave (at nominal 2.4 GHz)
}

template <int OP>
void report(const char* name, const uint32_t* din, uint32_t* dout) {
  // throughput: 8 waves/SIMD (2048 blocks x 256 thr on 256 CUs), 8 chains; latency: 1 wave/SIMD, 1 chain
  double t = run<OP, 8>(256 * 8, 2048, din, dout);   // cycles per wave-instr, 8 waves share a SIMD
  double l = run<OP, 1>(256, 8192, din, dout);       // one wave per SIMD, dependent chain
  printf("%-16s  SIMD cycles/instr (8 waves): %5.2f   dependent-chain cycles/instr (1 wave): %5.2f\n",
         name, t / 8.0, l);
}

int main() {
  uint32_t h[8] = {0x00FF1005u, 0x40302010u, 0x05000A03u, 0x0C0C0504u, 1, 2, 3, 4};
  uint32_t *din, *dout;
  (void)hipMalloc(&din, 64); (void)hipMalloc(&dout, 256 * 8 * 256 * 4);
  (void)hipMemcpy(din, h, 32, hipMemcpyHostToDevice);
  report<0>("v_sad_u8", din, dout);
  report<1>("v_sad_hi_u8", din, dout);
  report<9>("v_msad_u8", din, dout);
  report<2>("v_perm_b32", din, dout);
  report<3>("v_min3_u32", din, dout);
  report<10>("v_min_u32", din, dout);
  report<4>("v_add_u32", din, dout);
  report<5>("v_sub_u32", din, dout);
  report<6>("v_pk_add_u16", din, dout);
  report<7>("v_alignbyte", din, dout);
  report<8>("v_and_or_b32", din, dout);
  return 0;
}
