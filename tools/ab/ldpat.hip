// Microbenchmark: K1's cube load pattern vs channel pitch (timing experiment only).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>
#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("err %s line %d\n", hipGetErrorString(e), __LINE__); return 1; } } while (0)
constexpr int C = 16, N = 4096, P = 128, NT = 8, F = 4;
__global__ __launch_bounds__(512) void k1like(const float2* __restrict__ base, size_t pitch, size_t cubestride, int ntiles, float* out) {
    const int f = blockIdx.y, tile = blockIdx.x;
    const float2* x = base + f * cubestride;
    const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6, grp = lane >> 4, col = lane & 15;
    float sink = 0.f;
    const int t0 = wv * 4;
    float4 xv[4][4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
        const int t = t0 + u, nl = t / 4, p = ((t & 3) << 5) + 2 * col;
        const int n = tile * NT + nl;
#pragma unroll
        for (int j = 0; j < 4; ++j) xv[u][j] = *reinterpret_cast<const float4*>(x + (size_t)(4 * j + grp) * pitch + (size_t)n * P + p);
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 4; ++j) sink += xv[u][j].x + xv[u][j].y + xv[u][j].z + xv[u][j].w;
    if (sink == 1.2345e-30f) out[threadIdx.x] = sink;
}
__global__ __launch_bounds__(256) void flat(const float4* __restrict__ x, size_t n4, float* out) {
    float s = 0.f;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n4; i += (size_t)gridDim.x * 256) { float4 v = x[i]; s += v.x + v.y + v.z + v.w; }
    if (s == 1.2345e-30f) out[threadIdx.x] = s;
}
int main() {
    const int ntiles = 379;   // x2 used samples / NT
    const size_t maxpitch = (size_t)N * P + 4096;
    const size_t cubestride = maxpitch * C;
    const int ncubes = 8;
    float2* d; float* o;
    CHK(hipMalloc(&d, cubestride * ncubes * sizeof(float2)));
    CHK(hipMemset(d, 0, cubestride * ncubes * sizeof(float2)));
    CHK(hipMalloc(&o, 4096));
    hipEvent_t a, b; CHK(hipEventCreate(&a)); CHK(hipEventCreate(&b));
    const size_t pads[] = {0, 64, 512, 1024, 2048};
    for (size_t pad : pads) {
        const size_t pitch = (size_t)N * P + pad;
        float best = 1e9;
        for (int rep = 0; rep < 40; ++rep) {
            const float2* base = d + (size_t)(rep % 2) * 4 * cubestride;
            CHK(hipEventRecord(a));
            hipLaunchKernelGGL(k1like, dim3(ntiles, F), dim3(512), 0, 0, base, pitch, cubestride, ntiles, o);
            CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
            float ms; CHK(hipEventElapsedTime(&ms, a, b)); if (rep > 2 && ms < best) best = ms;
        }
        const double bytes = (double)F * ntiles * NT * C * P * 8;
        printf("pad %5zu: %.1f us  %.2f TB/s\n", pad, best * 1e3, bytes / (best * 1e-3) / 1e12);
    }
    {
        const size_t n4 = (size_t)F * 379 * NT * C * P * 8 / 16;
        for (int grid : {1024, 2048, 4096, 8192}) {
            float best = 1e9;
            for (int rep = 0; rep < 40; ++rep) {
                CHK(hipEventRecord(a));
                hipLaunchKernelGGL(flat, dim3(grid), dim3(256), 0, 0, (const float4*)(d + (size_t)(rep % 2) * 4 * cubestride), n4, o);
                CHK(hipEventRecord(b)); CHK(hipEventSynchronize(b));
                float ms; CHK(hipEventElapsedTime(&ms, a, b)); if (rep > 2 && ms < best) best = ms;
            }
            printf("flat grid %d: %.1f us  %.2f TB/s\n", grid, best * 1e3, n4 * 16.0 / (best * 1e-3) / 1e12);
        }
    }
    return 0;
}
