// Occupancy (workgroups per CU) of a 256-thread kernel vs its dynamic LDS size: finds the LDS
// allocation granularity the runtime applies on this device.
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ void __launch_bounds__(256) k(int* o) {
    extern __shared__ int s[];
    s[threadIdx.x] = threadIdx.x;
    __syncthreads();
    o[threadIdx.x] = s[255 - threadIdx.x];
}
int main() {
    int prev = -1;
    for (int b = 40000; b <= 82000; b += 64) {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, k, 256, b) != hipSuccess) return 1;
        if (n != prev) { printf("lds %d bytes -> %d workgroups/CU\n", b, n); prev = n; }
    }
    return 0;
}
