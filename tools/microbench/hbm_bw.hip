// Achievable HBM bandwidth on this MI355X for the access shapes of the staged kernels:
// 16-B loads (read-only reduction), 16-B nontemporal / plain stores (write-only), 16-B copy,
// on a 1 GiB buffer (4x the 256 MiB Infinity Cache).  Reports GB/s and the fraction of 8 TB/s.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>

typedef unsigned int u32x4 __attribute__((ext_vector_type(4)));

template <int UNROLL, bool NT>
__global__ __launch_bounds__(256) void rd(const u32x4* __restrict__ p, size_t n, uint32_t* out) {
    const size_t stride = (size_t)gridDim.x * 256;
    u32x4 acc = {0, 0, 0, 0};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride * UNROLL) {
        u32x4 v[UNROLL];
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) {
            const size_t j = i + u * stride;
            if (j < n) v[u] = NT ? __builtin_nontemporal_load(p + j) : p[j];
            else v[u] = acc;
        }
#pragma unroll
        for (int u = 0; u < UNROLL; ++u) acc ^= v[u];
    }
    if ((acc.x ^ acc.y ^ acc.z ^ acc.w) == 0x12345678u) out[0] = 1;
}

template <bool NT>
__global__ __launch_bounds__(256) void wr(u32x4* __restrict__ p, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256;
    const u32x4 v = {threadIdx.x, blockIdx.x, 1, 2};
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride) {
        if (NT) __builtin_nontemporal_store(v, p + i);
        else p[i] = v;
    }
}

__global__ __launch_bounds__(256) void cp(const u32x4* __restrict__ a, u32x4* __restrict__ b, size_t n) {
    const size_t stride = (size_t)gridDim.x * 256;
    for (size_t i = (size_t)blockIdx.x * 256 + threadIdx.x; i < n; i += stride * 4) {
        u32x4 v[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) v[u] = i + u * stride < n ? __builtin_nontemporal_load(a + i + u * stride) : v[0];
#pragma unroll
        for (int u = 0; u < 4; ++u)
            if (i + u * stride < n) __builtin_nontemporal_store(v[u], b + i + u * stride);
    }
}

template <class F>
void timeit(const char* name, double bytes, F f) {
    hipEvent_t e0, e1;
    (void)hipEventCreate(&e0);
    (void)hipEventCreate(&e1);
    f();
    f();
    (void)hipDeviceSynchronize();
    (void)hipEventRecord(e0);
    const int n = 10;
    for (int i = 0; i < n; ++i) f();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    const double gbs = bytes * n / (ms * 1e-3) / 1e9;
    printf("%-40s %8.1f GB/s  %.3f of 8 TB/s\n", name, gbs, gbs / 8000.0);
}

int main() {
    const size_t bytes = (size_t)1 << 30, n = bytes / 16;
    u32x4 *a, *b;
    uint32_t* o;
    (void)hipMalloc(&a, bytes);
    (void)hipMalloc(&b, bytes);
    (void)hipMalloc(&o, 64);
    (void)hipMemset(a, 1, bytes);
    (void)hipMemset(b, 2, bytes);
    for (int blocks : {1024, 2048, 4096, 8192}) {
        char nm[64];
        snprintf(nm, sizeof nm, "read 16B x4 unroll, %d blocks", blocks);
        timeit(nm, bytes, [&] { rd<4, false><<<blocks, 256>>>(a, n, o); });
        snprintf(nm, sizeof nm, "read 16B nt x8 unroll, %d blocks", blocks);
        timeit(nm, bytes, [&] { rd<8, true><<<blocks, 256>>>(a, n, o); });
        snprintf(nm, sizeof nm, "write 16B nt, %d blocks", blocks);
        timeit(nm, bytes, [&] { wr<true><<<blocks, 256>>>(b, n); });
        snprintf(nm, sizeof nm, "write 16B plain, %d blocks", blocks);
        timeit(nm, bytes, [&] { wr<false><<<blocks, 256>>>(b, n); });
        snprintf(nm, sizeof nm, "copy 16B nt (r+w bytes), %d blocks", blocks);
        timeit(nm, 2.0 * bytes, [&] { cp<<<blocks, 256>>>(a, b, n); });
    }
    return 0;
}
