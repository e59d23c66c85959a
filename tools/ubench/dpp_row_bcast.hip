// Checks v_mov_b32_dpp / v_mov_b64_dpp row_newbcast:k on gfx950: every lane of a 16-lane row
// should receive lane k of its row. Prints mismatches per (width, k).
#include <hip/hip_runtime.h>
#include <cstdio>

template <int K>
__global__ void k32(int* out)
{
    const int v = 1000 + (int)threadIdx.x;
    out[threadIdx.x] = __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xf, 0xf, false);
}
template <int K>
__global__ void k64(double* out)
{
    const double v = 1000.0 + threadIdx.x;
    out[threadIdx.x] = __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xf, 0xf, false);
}
// divergent: only row 1 and 3 active
template <int K>
__global__ void k32d(int* out)
{
    const int v = 1000 + (int)threadIdx.x;
    int r = -1;
    if ((threadIdx.x >> 4) & 1) r = __builtin_amdgcn_mov_dpp(v, 0x150 + K, 0xf, 0xf, false);
    out[threadIdx.x] = r;
}

template <int K>
int check()
{
    int* di;
    double* dd;
    hipMalloc(&di, 64 * sizeof(int));
    hipMalloc(&dd, 64 * sizeof(double));
    int hi[64];
    double hd[64];
    int bad32 = 0, bad64 = 0, badd = 0;
    hipLaunchKernelGGL(k32<K>, dim3(1), dim3(64), 0, 0, di);
    hipMemcpy(hi, di, sizeof(hi), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l++) bad32 += hi[l] != 1000 + (l & ~15) + K;
    hipLaunchKernelGGL(k64<K>, dim3(1), dim3(64), 0, 0, dd);
    hipMemcpy(hd, dd, sizeof(hd), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l++) bad64 += hd[l] != 1000.0 + (l & ~15) + K;
    hipLaunchKernelGGL(k32d<K>, dim3(1), dim3(64), 0, 0, di);
    hipMemcpy(hi, di, sizeof(hi), hipMemcpyDeviceToHost);
    for (int l = 0; l < 64; l++) badd += (((l >> 4) & 1) ? hi[l] != 1000 + (l & ~15) + K : hi[l] != -1);
    printf("row_newbcast:%d  b32 mismatches %d  b64 mismatches %d  b32 divergent mismatches %d  (lane 5: %d)\n", K,
           bad32, bad64, badd, hi[5]);
    hipFree(di);
    hipFree(dd);
    return bad32 + bad64 + badd;
}

int main()
{
    int bad = check<0>() + check<3>() + check<15>();
    printf(bad ? "MISMATCH\n" : "all lanes agree\n");
    return 0;
}
