// Column-block read bandwidth vs grid row pitch (probe for the fused FFT
// column passes): 8192 rows x 5440 columns of float2, workgroups of 64
// columns x 64 rows as k_cols_b_grid (contiguous rows) or k_cols_b_image
// (rows 128 apart), row pitch 8192 (power of two) or padded.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

template<int STRIDE>
__global__ __launch_bounds__(256) void k_read(const float2* __restrict__ g,
        size_t pitch, float* __restrict__ out, int M)
{
    const int c = threadIdx.x % 64, p = threadIdx.x / 64;
    const int k2 = blockIdx.x;
    const int ncb = (M + 63) / 64;
    float acc = 0.0f;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int col = cb * 64 + c;
        if (col >= M) continue;
        float2 v[16];
#pragma unroll
        for (int e = 0; e < 16; ++e)
        {
            const int row = STRIDE == 1 ? 64 * k2 + p + 4 * e
                                        : k2 + 128 * (p + 4 * e);
            v[e] = g[(size_t)row * pitch + col];
        }
#pragma unroll
        for (int e = 0; e < 16; ++e) acc += v[e].x + v[e].y;
    }
    out[blockIdx.x * 256 * gridDim.y + blockIdx.y * 256 + threadIdx.x] = acc;
}

int main()
{
    const int G = 8192, M = 5440;
    const size_t pitches[] = {8192, 8192 + 16, 8192 + 64, 8192 + 256};
    float2* g; float* out;
    hipMalloc(&g, (size_t)G * (8192 + 256) * sizeof(float2));
    hipMemset(g, 0, (size_t)G * (8192 + 256) * sizeof(float2));
    hipMalloc(&out, 128 * 64 * 256 * sizeof(float));
    hipEvent_t a, b;
    hipEventCreate(&a); hipEventCreate(&b);
    for (int pattern = 0; pattern < 2; ++pattern)
        for (size_t pitch : pitches)
            for (int split : {12, 24})
            {
                dim3 grid(128, split);
                float best = 1e9f;
                for (int rep = 0; rep < 6; ++rep)
                {
                    hipEventRecord(a);
                    if (pattern == 0) k_read<1><<<grid, 256>>>(g, pitch, out, M);
                    else k_read<128><<<grid, 256>>>(g, pitch, out, M);
                    hipEventRecord(b);
                    hipEventSynchronize(b);
                    float ms; hipEventElapsedTime(&ms, a, b);
                    if (rep > 0 && ms < best) best = ms;
                }
                const double bytes = (double)G * M * 8;
                printf("pattern %s pitch %zu split %d: %.1f us, %.2f TB/s\n",
                        pattern == 0 ? "contig-rows" : "rows-128-apart",
                        pitch, split, best * 1e3, bytes / (best * 1e-3) / 1e12);
            }
    return 0;
}
