// Issue rates of the VALU ops a guided-filter / box-SAD kernel is built from (gfx950, wave64).
// 8 independent chains per thread, 8 waves per SIMD (256-thread blocks, 8 blocks per CU), every
// instruction written as inline asm so the measured opcode is exactly the named one.
// Output: SIMD cycles per wave-instruction at the 2.4 GHz nominal clock.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

#define OP2(name, asmstr)                                                                     \
    struct name {                                                                             \
        static constexpr const char* s = #asmstr;                                             \
        __device__ static void run(uint32_t& a, uint32_t x) { asm volatile(#asmstr " %0, %0, %1" : "+v"(a) : "v"(x)); } \
    };
#define OP3(name, asmstr)                                                                     \
    struct name {                                                                             \
        static constexpr const char* s = #asmstr;                                             \
        __device__ static void run(uint32_t& a, uint32_t x) { asm volatile(#asmstr " %0, %0, %1, %0" : "+v"(a) : "v"(x)); } \
    };
#define OP1(name, asmstr)                                                                     \
    struct name {                                                                             \
        static constexpr const char* s = #asmstr;                                             \
        __device__ static void run(uint32_t& a, uint32_t x) { asm volatile(#asmstr " %0, %1" : "=v"(a) : "v"(x ^ a)); } \
    };

OP2(Add, v_add_u32)
OP2(AddF, v_add_f32)
OP2(MulF, v_mul_f32)
OP3(FmaF, v_fma_f32)
OP2(MinF, v_min_f32)
OP2(MinI, v_min_i32)
OP2(MulU24, v_mul_u32_u24)
OP2(MulI24, v_mul_i32_i24)
OP3(MadU24, v_mad_u32_u24)
OP3(MadI24, v_mad_i32_i24)
OP3(Sad, v_sad_u8)
OP3(Perm, v_perm_b32)
OP3(LshlAdd, v_lshl_add_u32)
OP3(LshlOr, v_lshl_or_b32)
OP3(Add3, v_add3_u32)
OP3(Bfe, v_bfe_u32)
OP3(Min3F, v_min3_f32)
OP3(Min3I, v_min3_i32)
OP2(Lshr, v_lshrrev_b32)
OP2(MulLo, v_mul_lo_u32)
OP1(CvtFI, v_cvt_f32_i32)
OP1(CvtFU, v_cvt_f32_u32)
OP1(CvtFUb, v_cvt_f32_ubyte1)
OP1(CvtIF, v_cvt_i32_f32)
OP1(Rcp, v_rcp_f32)

struct CndMask {
    static constexpr const char* s = "v_cmp_lt_f32 + v_cndmask_b32";
    __device__ static void run(uint32_t& a, uint32_t x) {
        asm volatile("v_cmp_lt_f32 vcc, %0, %1\n\tv_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(x) : "vcc");
    }
};
struct CndOnly {
    static constexpr const char* s = "v_cndmask_b32 (vcc const)";
    __device__ static void run(uint32_t& a, uint32_t x) {
        asm volatile("v_cndmask_b32 %0, %0, %1, vcc" : "+v"(a) : "v"(x) : "vcc");
    }
};
// packed f32: a 64-bit register pair per chain, so 8 chains = 16 VGPRs
struct PkAdd {
    static constexpr const char* s = "v_pk_add_f32";
    static constexpr bool pk = true;
    __device__ static void run2(uint64_t& a, uint64_t x) { asm volatile("v_pk_add_f32 %0, %0, %1" : "+v"(a) : "v"(x)); }
};
struct PkMul {
    static constexpr const char* s = "v_pk_mul_f32";
    static constexpr bool pk = true;
    __device__ static void run2(uint64_t& a, uint64_t x) { asm volatile("v_pk_mul_f32 %0, %0, %1" : "+v"(a) : "v"(x)); }
};
struct PkFma {
    static constexpr const char* s = "v_pk_fma_f32";
    static constexpr bool pk = true;
    __device__ static void run2(uint64_t& a, uint64_t x) { asm volatile("v_pk_fma_f32 %0, %0, %1, %0" : "+v"(a) : "v"(x)); }
};
struct AddU64 {
    static constexpr const char* s = "v_lshl_add_u64";
    static constexpr bool pk = true;
    __device__ static void run2(uint64_t& a, uint64_t x) { asm volatile("v_lshl_add_u64 %0, %1, 0, %0" : "+v"(a) : "v"(x)); }
};

template <class O, class = void> struct IsPk { static constexpr bool v = false; };
template <class O> struct IsPk<O, decltype((void)O::pk)> { static constexpr bool v = O::pk; };

template <class O>
__global__ __launch_bounds__(256) void thr(const uint32_t* in, uint32_t* out, int iters) {
    uint32_t s = 0;
    if constexpr (IsPk<O>::v) {
        uint64_t xs[8], acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            xs[c] = ((uint64_t)in[(threadIdx.x + c) & 7] << 32) | in[(threadIdx.x + c + 1) & 7];
            acc[c] = ((uint64_t)(threadIdx.x * 7 + c) << 32) | (threadIdx.x + c);
        }
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < 8; ++c) O::run2(acc[c], xs[(c + k) & 7]);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) s += (uint32_t)acc[c] ^ (uint32_t)(acc[c] >> 32);
    } else {
        uint32_t xs[8], acc[8];
#pragma unroll
        for (int c = 0; c < 8; ++c) {
            xs[c] = in[(threadIdx.x + c) & 7] + c;
            acc[c] = threadIdx.x * 7 + c;
        }
        for (int i = 0; i < iters; ++i) {
#pragma unroll
            for (int k = 0; k < 8; ++k)
#pragma unroll
                for (int c = 0; c < 8; ++c) O::run(acc[c], xs[(c + k) & 7]);
        }
#pragma unroll
        for (int c = 0; c < 8; ++c) s += acc[c];
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = s;
}

template <class O> void report(const uint32_t* din, uint32_t* dout, int nops = 1) {
    const int blocks = 256 * 8, iters = 512;
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    thr<O><<<blocks, 256>>>(din, dout, iters);
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) thr<O><<<blocks, 256>>>(din, dout, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    // per SIMD: 8 waves x iters * 64 instructions (x nops asm instructions each)
    const double cyc = ms * 1e-3 * 2.4e9 / (8.0 * iters * 64 * nops);
    printf("%-34s SIMD cycles per wave-instr: %5.2f\n", O::s, cyc);
}

int main() {
    uint32_t h[8] = {0x3F800001u, 0x40302010u, 0x05000A03u, 0x0C0C0504u, 0x3F000000u, 2, 3, 4};
    uint32_t *din, *dout;
    (void)hipMalloc(&din, 64);
    (void)hipMalloc(&dout, 256 * 8 * 256 * 4);
    (void)hipMemcpy(din, h, 32, hipMemcpyHostToDevice);
    report<Add>(din, dout);
    report<AddF>(din, dout);
    report<MulF>(din, dout);
    report<FmaF>(din, dout);
    report<MinF>(din, dout);
    report<MinI>(din, dout);
    report<PkAdd>(din, dout);
    report<PkMul>(din, dout);
    report<PkFma>(din, dout);
    report<AddU64>(din, dout);
    report<MulU24>(din, dout);
    report<MulI24>(din, dout);
    report<MadU24>(din, dout);
    report<MadI24>(din, dout);
    report<MulLo>(din, dout);
    report<Sad>(din, dout);
    report<Perm>(din, dout);
    report<LshlAdd>(din, dout);
    report<LshlOr>(din, dout);
    report<Add3>(din, dout);
    report<Bfe>(din, dout);
    report<Min3F>(din, dout);
    report<Min3I>(din, dout);
    report<Lshr>(din, dout);
    report<CvtFI>(din, dout);
    report<CvtFU>(din, dout);
    report<CvtFUb>(din, dout);
    report<CvtIF>(din, dout);
    report<Rcp>(din, dout);
    report<CndOnly>(din, dout);
    report<CndMask>(din, dout, 2);
    return 0;
}
