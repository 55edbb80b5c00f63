// Operand layout and issue rate of v_mfma_f32_4x4x1_16b_f32 on gfx950
// (probe for a 4-visibility-granular k_tower_idft). Part 1: for each lane
// p, A one-hot at lane p and B[q] = q + 1; every nonzero C[l][r] = B[q]
// names one product A[p] * B[q] landing in lane l, register r. Part 2:
// cycles per instruction for back-to-back 4x4x1_16b and 16x16x4 (eight
// independent accumulators, one wave).
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

using f32x4 = __attribute__((ext_vector_type(4))) float;

__global__ void k_layout(float* out)
{
    const int p = blockIdx.x, l = threadIdx.x;
    const float a = (l == p) ? 1.0f : 0.0f;
    const float b = (float)(l + 1);
    f32x4 c = {0.0f, 0.0f, 0.0f, 0.0f};
    c = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; ++r) out[(p * 64 + l) * 4 + r] = c[r];
}

template<int KIND>
__global__ void k_rate(float* out, long long* cyc, int iters)
{
    const int l = threadIdx.x;
    float a = 1.0f + l * 1e-3f, b = 1.0f - l * 1e-3f;
    f32x4 c0 = {0, 0, 0, 0}, c1 = c0, c2 = c0, c3 = c0;
    f32x4 c4 = c0, c5 = c0, c6 = c0, c7 = c0;
    const long long t0 = clock64();
    for (int i = 0; i < iters; ++i)
    {
        if (KIND == 0)
        {
            c0 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, b, c3, 0, 0, 0);
            c4 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, b, c4, 0, 0, 0);
            c5 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, a, c5, 0, 0, 0);
            c6 = __builtin_amdgcn_mfma_f32_4x4x1f32(a, a, c6, 0, 0, 0);
            c7 = __builtin_amdgcn_mfma_f32_4x4x1f32(b, b, c7, 0, 0, 0);
        }
        else
        {
            c0 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c0, 0, 0, 0);
            c1 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c1, 0, 0, 0);
            c2 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c2, 0, 0, 0);
            c3 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c3, 0, 0, 0);
            c4 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, c4, 0, 0, 0);
            c5 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, a, c5, 0, 0, 0);
            c6 = __builtin_amdgcn_mfma_f32_16x16x4f32(a, a, c6, 0, 0, 0);
            c7 = __builtin_amdgcn_mfma_f32_16x16x4f32(b, b, c7, 0, 0, 0);
        }
    }
    const long long t1 = clock64();
    out[l] = c0[0] + c1[1] + c2[2] + c3[3] + c4[0] + c5[1] + c6[2] + c7[3];
    if (l == 0) cyc[0] = t1 - t0;
}

int main()
{
    float* d_out;
    long long* d_cyc;
    hipMalloc(&d_out, 64 * 64 * 4 * sizeof(float));
    hipMalloc(&d_cyc, sizeof(long long));
    k_layout<<<64, 64>>>(d_out);
    std::vector<float> h(64 * 64 * 4);
    hipMemcpy(h.data(), d_out, h.size() * sizeof(float), hipMemcpyDeviceToHost);
    // For each A lane p: the (C lane, reg, B lane) products it feeds.
    for (int p = 0; p < 64; ++p)
    {
        printf("A%02d:", p);
        for (int l = 0; l < 64; ++l)
            for (int r = 0; r < 4; ++r)
            {
                const float v = h[(p * 64 + l) * 4 + r];
                if (v != 0.0f) printf(" C[%d][%d]=B%d", l, r, (int)v - 1);
            }
        printf("\n");
    }
    const int iters = 4096;
    for (int kind = 0; kind < 2; ++kind)
    {
        long long cyc = 0;
        for (int rep = 0; rep < 3; ++rep)
        {
            if (kind == 0) k_rate<0><<<1, 64>>>(d_out, d_cyc, iters);
            else k_rate<1><<<1, 64>>>(d_out, d_cyc, iters);
            hipMemcpy(&cyc, d_cyc, sizeof(cyc), hipMemcpyDeviceToHost);
        }
        printf("%s: %.2f clock64 ticks per instruction\n",
                kind == 0 ? "4x4x1_16b" : "16x16x4", (double)cyc / (8.0 * iters));
    }
    return 0;
}
