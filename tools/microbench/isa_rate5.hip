// Issue cost of the multi-SAD instructions for the box kernel's phase V:
// v_qsad_pk_u16_u8 (4 byte-SADs of shifted windows, 16-bit accumulate, 64-bit D) and v_mqsad_u32_u8
// (4 masked byte-SADs, 32-bit accumulate, 128-bit D), beside v_sad_u8 as the baseline.
// 8 independent chains per thread, 8 waves per SIMD, inline asm so the opcode is exactly the named
// one; output: SIMD cycles per wave-instruction at the 2.4 GHz nominal clock (as isa_rate4.hip).
#include <hip/hip_runtime.h>
#include <cstdint>
#include <cstdio>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int OP>
__global__ __launch_bounds__(256) void thr(const uint32_t* in, uint32_t* out, int iters) {
    uint32_t s = 0;
    uint64_t src[8];
#pragma unroll
    for (int c = 0; c < 8; ++c) src[c] = ((uint64_t)in[(threadIdx.x + c) & 7] << 32) | in[(threadIdx.x + c + 3) & 7];
    const uint32_t ref = in[threadIdx.x & 7];
    if constexpr (OP == 0) {          // v_sad_u8
        uint32_t acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = threadIdx.x + c;
        for (int i = 0; i < iters; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < 8; ++c) asm volatile("v_sad_u8 %0, %1, %2, %0" : "+v"(acc[c]) : "v"((uint32_t)src[c]), "v"(ref));
#pragma unroll
        for (int c = 0; c < 8; ++c) s ^= acc[c];
    } else if constexpr (OP == 1) {   // v_qsad_pk_u16_u8
        uint64_t acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = threadIdx.x + c;
        for (int i = 0; i < iters; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < 8; ++c) asm volatile("v_qsad_pk_u16_u8 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(src[c]), "v"(ref));
#pragma unroll
        for (int c = 0; c < 8; ++c) s ^= (uint32_t)acc[c] ^ (uint32_t)(acc[c] >> 32);
    } else {                          // v_mqsad_u32_u8
        u32x4 acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) acc[c] = u32x4{threadIdx.x, (uint32_t)c, 1u, 2u};
        for (int i = 0; i < iters; ++i)
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < 8; ++c) asm volatile("v_mqsad_u32_u8 %0, %1, %2, %0" : "+v"(acc[c]) : "v"(src[c]), "v"(ref));
#pragma unroll
        for (int c = 0; c < 8; ++c) s ^= acc[c].x ^ acc[c].y ^ acc[c].z ^ acc[c].w;
    }
    if (s == 0x12345678u) out[0] = s;
}

template <int OP>
void report(const char* name, const uint32_t* din, uint32_t* dout) {
    const int iters = 2048, blocks = 256 * 8;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    thr<OP><<<blocks, 256>>>(din, dout, 16);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    thr<OP><<<blocks, 256>>>(din, dout, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    // per SIMD: 8 waves x iters x 64 instructions
    const double inst = 8.0 * iters * 64;
    printf("%-22s SIMD cycles per wave-instr: %6.2f\n", name, ms * 1e-3 * 2.4e9 / inst);
}

int main() {
    uint32_t *din, *dout;
    (void)hipMalloc(&din, 64);
    (void)hipMalloc(&dout, 64);
    uint32_t h[8] = {0x01020304u, 0x11223344u, 0x80706050u, 0xFFEEDDCCu, 0x0A0B0C0Du, 0x7F7F7F7Fu, 0x10203040u, 0x55AA55AAu};
    (void)hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    report<0>("v_sad_u8", din, dout);
    report<1>("v_qsad_pk_u16_u8", din, dout);
    report<2>("v_mqsad_u32_u8", din, dout);
    return 0;
}
