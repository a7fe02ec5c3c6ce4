#include <hip/hip_runtime.h>
#include <cstdio>
__device__ __forceinline__ int lo1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xA0, 0xF, 0xF, false); }
__device__ __forceinline__ int hi1(int v) { return __builtin_amdgcn_update_dpp(0, v, 0xF5, 0xF, 0xF, false); }
__device__ __forceinline__ int lo4(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x114, 0xF, 0xA, false); }
__device__ __forceinline__ int hi4(int v) { return __builtin_amdgcn_update_dpp(v, v, 0x104, 0xF, 0x5, false); }
__global__ void k(const int* in, int* out)
{
    const int l = threadIdx.x;
    int v = in[l], w = in[64 + l];
    int a = lo1(v), b = hi1(v), c = lo4(w), d = hi4(w);
    int e = hi1(v) + lo1(v), f = lo1(v) - hi1(v);      // combinable forms
    out[l] = a; out[64 + l] = b; out[128 + l] = c; out[192 + l] = d; out[256 + l] = e; out[320 + l] = f;
}
int main()
{
    int h[128], o[384]; for (int i = 0; i < 128; ++i) h[i] = 1000 + i * 7;
    int *din, *dout; hipMalloc(&din, sizeof h); hipMalloc(&dout, sizeof o);
    hipMemcpy(din, h, sizeof h, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(1), dim3(64), 0, 0, din, dout);
    hipMemcpy(o, dout, sizeof o, hipMemcpyDeviceToHost);
    int bad = 0;
    for (int l = 0; l < 64; ++l) {
        int v = h[l], lo = h[l & ~1], hi = h[l | 1];
        int c = h[64 + (l & ~4)], d = h[64 + (l | 4)];
        int exp[6] = {lo, hi, c, d, hi + lo, lo - hi};
        for (int t = 0; t < 6; ++t) if (o[64 * t + l] != exp[t]) { if (bad < 20) printf("lane %d test %d got %d want %d (v %d)\n", l, t, o[64 * t + l], exp[t], v); ++bad; }
    }
    printf("bad %d\n", bad);
    return bad != 0;
}
