// Pruned, fused 2-D FFT passes of the ES (de)gridder. See es_fft.h.
//
// Building block: a length-L Stockham FFT (natural order in and out) shared
// by P threads of a workgroup, EPT = L / P elements per thread, two or three
// stages of radix <= 32. Each stage is an in-register DFT (radix-2
// butterflies with compile-time roots of unity) preceded by the stage's
// twiddles; stages exchange data through LDS. Twiddles depend only on the
// thread's lane, so each workgroup reads them once from the G-entry table
// and keeps them in registers while it loops over rows / column blocks.
//
// Row passes: one workgroup per row at a time, LDS index e + e/16 (padding
// breaks the stride-16 bank pattern of the first stage's stores).
// Column passes: B = 256 / P adjacent columns per workgroup (B * 8 bytes
// contiguous per row access: 256 B at L = 128, 512 B at L = 64), LDS index
// e * B + column.
#include <algorithm>
#include <climits>
#include <cstdlib>
#include <cmath>
#include <type_traits>
#include <utility>
#include <vector>

#include "es_fft.h"
#include "es_fft_wstack.h"
#include "es_image_dev.h"
#include "../utility/sdp_hip.h"

// Waves per SIMD of the column passes (VGPR budget). Column pass A and
// the degrid image pass fit 128 VGPRs without spills at 4 (3 at 131-132
// VGPRs): config 2 gridding 7382 -> 7466 Mvis/s (FFT phase 0.310 -> 0.314
// ms, image phase 0.171 -> 0.151 ms), degridding 6362 -> 6389 (A/B, three
// alternating rounds on one box). Column pass B (149 VGPRs with the image
// values it adds to held across the transform) spills at 4 (image phase
// 0.32 ms); loading those values after the transform instead (103 VGPRs,
// 4-5 waves) measured 0.164-0.175 ms.
#define SDP_COLA_WAVES 4
#define SDP_COLB_WAVES 3

namespace sdp_es {
namespace {

using img::phasor;

__device__ __forceinline__ float2 cadd(float2 a, float2 b)
{
    return make_float2(a.x + b.x, a.y + b.y);
}

__device__ __forceinline__ float2 csub(float2 a, float2 b)
{
    return make_float2(a.x - b.x, a.y - b.y);
}

__device__ __forceinline__ float2 cmul(float2 a, float2 b)
{
    return make_float2(a.x * b.x - a.y * b.y, a.x * b.y + a.y * b.x);
}

// Compile-time roots of unity ----------------------------------------------

constexpr double kTwoPi = 6.283185307179586476925286766559;

// Taylor series, |x| <= pi: terms fall below 1e-20 well before n = 20.
constexpr double cx_sin(double x)
{
    double t = x, s = x;
    for (int n = 1; n < 20; ++n)
    {
        t *= -x * x / ((2.0 * n) * (2.0 * n + 1.0));
        s += t;
    }
    return s;
}

constexpr double cx_cos(double x)
{
    double t = 1.0, s = 1.0;
    for (int n = 1; n < 20; ++n)
    {
        t *= -x * x / ((2.0 * n - 1.0) * (2.0 * n));
        s += t;
    }
    return s;
}

constexpr double root_angle(int m, int r)
{
    const double a = kTwoPi * m / r;
    return (a > kTwoPi / 2) ? a - kTwoPi : a;
}

constexpr int bit_reverse(int i, int r)
{
    int o = 0;
    for (int b = 1; b < r; b <<= 1)
    {
        o = (o << 1) | (i & 1);
        i >>= 1;
    }
    return o;
}

template<int I, int R>
constexpr int kBitRev = bit_reverse(I, R);

// b * exp(SIGN * 2 pi i * M / R), trivial rotations without multiplies.
template<int SIGN, int M, int R>
__device__ __forceinline__ float2 rotate(float2 b)
{
    if constexpr (M == 0)
        return b;
    else if constexpr (2 * M == R)
        return make_float2(-b.x, -b.y);
    else if constexpr (4 * M == R)
        return SIGN > 0 ? make_float2(-b.y, b.x) : make_float2(b.y, -b.x);
    else if constexpr (4 * M == 3 * R)
        return SIGN > 0 ? make_float2(b.y, -b.x) : make_float2(-b.y, b.x);
    else
    {
        constexpr float c = (float)cx_cos(root_angle(M, R));
        constexpr float s = (float)(SIGN * cx_sin(root_angle(M, R)));
        return make_float2(b.x * c - b.y * s, b.x * s + b.y * c);
    }
}

template<int SIGN, int R, int HALF, int IDX>
__device__ __forceinline__ void butterfly(float2* t)
{
    constexpr int I = (IDX / HALF) * 2 * HALF;
    constexpr int K = IDX % HALF;
    constexpr int M = K * (R / (2 * HALF));
    const float2 a = t[I + K];
    const float2 b = rotate<SIGN, M, R>(t[I + K + HALF]);
    t[I + K] = cadd(a, b);
    t[I + K + HALF] = csub(a, b);
}

template<int SIGN, int R, int HALF, int... IDX>
__device__ __forceinline__ void dft_level(float2* t,
        std::integer_sequence<int, IDX...>)
{
    (butterfly<SIGN, R, HALF, IDX>(t), ...);
}

template<int SIGN, int R, int HALF>
__device__ __forceinline__ void dft_levels(float2* t)
{
    if constexpr (HALF < R)
    {
        dft_level<SIGN, R, HALF>(t, std::make_integer_sequence<int, R / 2>{});
        dft_levels<SIGN, R, 2 * HALF>(t);
    }
}

template<int R, int... I>
__device__ __forceinline__ void bitrev_copy(float2* t, const float2* x,
        std::integer_sequence<int, I...>)
{
    ((t[kBitRev<I, R>] = x[I]), ...);
}

template<int R, int... I>
__device__ __forceinline__ void copy_back(float2* x, const float2* t,
        std::integer_sequence<int, I...>)
{
    ((x[I] = t[I]), ...);
}

// In-place R-point DFT of x[0..R): X[k] = sum_n x[n] exp(SIGN 2 pi i nk/R).
template<int SIGN, int R>
__device__ __forceinline__ void dft(float2* x)
{
    if constexpr (R > 1)
    {
        float2 t[R];
        bitrev_copy<R>(t, x, std::make_integer_sequence<int, R>{});
        dft_levels<SIGN, R, 1>(t);
        copy_back<R>(x, t, std::make_integer_sequence<int, R>{});
    }
}

// Stockham FFT of length L over P threads ----------------------------------
//
// Stage s (radix R, NS = product of earlier radices) maps butterfly j
// (j = p + q * P, q < EPT / R) from inputs j + r * L / R to outputs
// (j / NS) * NS * R + j % NS + r * NS, after multiplying input r by
// exp(SIGN 2 pi i r (j % NS) / (NS R)). First-stage inputs and last-stage
// outputs are exchanged with the caller through load / store functors.
template<int L, int P, int R0, int R1, int R2, int R3, int SIGN>
struct Fft
{
    static constexpr int EPT = L / P;
    static constexpr bool kThree = R2 > 1;
    static constexpr bool kFour = R3 > 1;
    static_assert(!kFour || kThree, "a fourth stage needs a third");
    static constexpr int NS1 = R0;
    static constexpr int NS2 = R0 * R1;
    static constexpr int NS3 = R0 * R1 * R2;
    static constexpr int RL = kFour ? R3 : (kThree ? R2 : R1);
    static_assert(R0 * R1 * (kThree ? R2 : 1) * (kFour ? R3 : 1) == L,
            "radices must multiply to L");
    static_assert(EPT % R0 == 0 && EPT % R1 == 0 && (!kThree || EPT % R2 == 0)
            && (!kFour || EPT % R3 == 0),
            "each radix must divide the elements per thread");
    static_assert(R0 == 16, "first radix 16 (LDS layouts rely on it)");
    // Butterflies of one thread share the twiddles when P % NS == 0.
    static constexpr int TQ1 = (P % NS1 == 0) ? 1 : EPT / R1;
    static constexpr int TQ2 = kThree ? ((P % NS2 == 0) ? 1 : EPT / R2) : 1;
    static constexpr int TQ3 = kFour ? ((P % NS3 == 0) ? 1 : EPT / R3) : 1;

    // Stage twiddles w^r (w = exp(SIGN 2 pi i k / (NS R)), r < R) are kept
    // as two short tables, w^b (b < LO) and w^(a LO) (a < R / LO), both read
    // exactly from the double-derived table; w^r = w^(a LO) * w^b costs one
    // complex multiply (<= 1.5 ulp) and saves two thirds of the registers.
    template<int R>
    struct Split
    {
        static constexpr int LO = (R == 32) ? 8 : (R >= 8 ? 4 : R);
        static constexpr int HI = R / LO;
    };
    template<int R, int TQ>
    struct StageTw
    {
        float2 lo[TQ][Split<R>::LO > 1 ? Split<R>::LO - 1 : 1];
        float2 hi[TQ][Split<R>::HI > 1 ? Split<R>::HI - 1 : 1];
    };
    StageTw<R1, TQ1> tw1;
    StageTw<kThree ? R2 : 2, TQ2> tw2;
    StageTw<kFour ? R3 : 2, TQ3> tw3;

    // W[m] = exp(-2 pi i m / G); exp(SIGN 2 pi i a / b) = W^(a G / b)*.
    static __device__ __forceinline__ float2 twiddle(
            const float2* __restrict__ W, int m)
    {
        float2 w = W[m];
        if (SIGN > 0) w.y = -w.y;
        return w;
    }

    template<int R, int NS, int TQ>
    static __device__ __forceinline__ void init_stage(StageTw<R, TQ>& t,
            int p, const float2* __restrict__ W, int G)
    {
        constexpr int LO = Split<R>::LO, HI = Split<R>::HI;
        const int s = G / (NS * R);
#pragma unroll
        for (int q = 0; q < TQ; ++q)
        {
            const int k = (p + q * P) & (NS - 1);
#pragma unroll
            for (int b = 1; b < LO; ++b) t.lo[q][b - 1] = twiddle(W, b * k * s);
#pragma unroll
            for (int a = 1; a < HI; ++a)
                t.hi[q][a - 1] = twiddle(W, a * LO * k * s);
        }
    }

    __device__ __forceinline__ void init(int p, const float2* __restrict__ W,
            int G)
    {
        init_stage<R1, NS1, TQ1>(tw1, p, W, G);
        if constexpr (kThree) init_stage<R2, NS2, TQ2>(tw2, p, W, G);
        if constexpr (kFour) init_stage<R3, NS3, TQ3>(tw3, p, W, G);
    }

    // Called once per row / column block: makes the stored twiddles opaque
    // so that the hi * lo products are formed where used instead of being
    // hoisted out of the loop (which would need all R - 1 per stage live).
    template<class T>
    static __device__ __forceinline__ void opaque_all(T& t)
    {
        float* f = reinterpret_cast<float*>(&t);
#pragma unroll
        for (unsigned i = 0; i < sizeof(T) / sizeof(float); ++i)
            asm volatile("" : "+v"(f[i]));
    }

    __device__ __forceinline__ void refresh()
    {
        opaque_all(tw1);
        if constexpr (kThree) opaque_all(tw2);
        if constexpr (kFour) opaque_all(tw3);
    }

    // v[0..R) *= w^r.
    template<int R, int TQ>
    static __device__ __forceinline__ void apply_stage(float2* v,
            const StageTw<R, TQ>& t, int q)
    {
        constexpr int LO = Split<R>::LO;
        const int qq = (TQ == 1) ? 0 : q;
#pragma unroll
        for (int r = 1; r < R; ++r)
        {
            const int a = r / LO, b = r % LO;
            float2 w;
            if (a == 0) w = t.lo[qq][b - 1];
            else if (b == 0) w = t.hi[qq][a - 1];
            else w = cmul(t.hi[qq][a - 1], t.lo[qq][b - 1]);
            v[r] = cmul(v[r], w);
        }
    }

    // Element index held in output slot i after the transform is
    // p + out_const(i); input slot q * R0 + r holds p + q * P + r * L / R0.
    // Load / store functors get that constant part (the caller adds p), so
    // that every address is one per-thread base plus a uniform offset.
    static constexpr int out_const(int i)
    {
        return (i / RL) * P + (i % RL) * (L / RL);
    }

    static __device__ __forceinline__ int out_index(int p, int i)
    {
        return p + out_const(i);
    }

    template<class Load>
    static __device__ __forceinline__ void load_input(float2 (&v)[EPT], Load ld)
    {
#pragma unroll
        for (int q = 0; q < EPT / R0; ++q)
#pragma unroll
            for (int r = 0; r < R0; ++r)
                v[q * R0 + r] = ld(q * P + r * (L / R0));
    }

    template<class Store>
    static __device__ __forceinline__ void store_output(
            const float2 (&v)[EPT], Store st)
    {
#pragma unroll
        for (int i = 0; i < EPT; ++i) st(out_const(i), i, v[i]);
    }

    // Stage output (radix R, stride NS) -> LDS -> next stage input (radix
    // RN). Every LDS index is base(thread) + off(compile-time constant), so
    // each access is one ds op with an immediate offset and no per-element
    // address registers: the store position of butterfly j = p + q * P,
    // element r, splits as below when P % NS == 0 (j / NS and j % NS then
    // split over p and q) or when every j < NS.
    template<int R, int NS, int RN, class Idx>
    static __device__ __forceinline__ void exchange(float2 (&v)[EPT], int p,
            float2* lds, Idx idx)
    {
        constexpr bool kSplit = (P % NS) == 0;
        static_assert(kSplit || P * (EPT / R) <= NS, "unsupported stage shape");
        const int sbase = kSplit ? (p / NS) * NS * R + (p & (NS - 1)) : p;
        float2* st = lds + idx.base(sbase);
        __syncthreads();
#pragma unroll
        for (int q = 0; q < EPT / R; ++q)
#pragma unroll
            for (int r = 0; r < R; ++r)
                st[Idx::off(kSplit ? q * P * R + r * NS : q * P + r * NS)] =
                        v[q * R + r];
        __syncthreads();
        const float2* ld = lds + idx.base(p);
#pragma unroll
        for (int q = 0; q < EPT / RN; ++q)
#pragma unroll
            for (int r = 0; r < RN; ++r)
                v[q * RN + r] = ld[Idx::off(q * P + r * (L / RN))];
    }

    template<class Idx>
    __device__ __forceinline__ void transform(float2 (&v)[EPT], int p,
            float2* lds, Idx idx)
    {
        refresh();
#pragma unroll
        for (int q = 0; q < EPT / R0; ++q) dft<SIGN, R0>(&v[q * R0]);
        exchange<R0, 1, R1>(v, p, lds, idx);
#pragma unroll
        for (int q = 0; q < EPT / R1; ++q)
        {
            apply_stage<R1, TQ1>(&v[q * R1], tw1, q);
            dft<SIGN, R1>(&v[q * R1]);
        }
        if constexpr (kThree)
        {
            exchange<R1, NS1, R2>(v, p, lds, idx);
#pragma unroll
            for (int q = 0; q < EPT / R2; ++q)
            {
                apply_stage<R2, TQ2>(&v[q * R2], tw2, q);
                dft<SIGN, R2>(&v[q * R2]);
            }
        }
        if constexpr (kFour)
        {
            exchange<R2, NS2, R3>(v, p, lds, idx);
#pragma unroll
            for (int q = 0; q < EPT / R3; ++q)
            {
                apply_stage<R3, TQ3>(&v[q * R3], tw3, q);
                dft<SIGN, R3>(&v[q * R3]);
            }
        }
    }
};

// Row transform of length G: threads and radices.
template<int G> struct RowPlan;
template<> struct RowPlan<1024>  { static constexpr int P = 64,  R0 = 16, R1 = 16, R2 = 4, R3 = 1; };
template<> struct RowPlan<2048>  { static constexpr int P = 128, R0 = 16, R1 = 16, R2 = 8, R3 = 1; };
template<> struct RowPlan<4096>  { static constexpr int P = 256, R0 = 16, R1 = 16, R2 = 16, R3 = 1; };
#ifndef ES_ROW8K_P256
// 512 threads, 16 elements each: half the registers of the 256-thread
// three-stage plan, so the two workgroups an 8192-point row's LDS allows
// per CU bring 4 waves per SIMD instead of 2.
template<> struct RowPlan<8192>  { static constexpr int P = 512, R0 = 16, R1 = 8, R2 = 8, R3 = 8; };
#else
template<> struct RowPlan<8192>  { static constexpr int P = 256, R0 = 16, R1 = 16, R2 = 32, R3 = 1; };
#endif
template<> struct RowPlan<16384> { static constexpr int P = 512, R0 = 16, R1 = 32, R2 = 32, R3 = 1; };

template<int G, int SIGN>
using RowFft = Fft<G, RowPlan<G>::P, RowPlan<G>::R0, RowPlan<G>::R1,
        RowPlan<G>::R2, RowPlan<G>::R3, SIGN>;

constexpr size_t row_lds_bytes(int G)
{
    return (size_t)(G + G / 16) * sizeof(float2);
}

// Column transform of length L: 16 elements per thread, 256 threads.
template<int L>
struct ColPlan
{
    static constexpr int P = L / 16;
    static constexpr int B = 256 / P;      // columns per workgroup
};

template<int L, int SIGN>
using ColFft = Fft<L, ColPlan<L>::P, 16, L / 16, 1, 1, SIGN>;

constexpr size_t kColLdsBytes = 4096 * sizeof(float2);   // L * B = 4096

// LDS layouts. idx(b + c) == base(b) + off(c) for the bases and constant
// offsets Fft::exchange forms.
//
// Rows: element e at e + e / 16 (one pad slot per 16): the first stage's
// stride-16 stores then hit 32 distinct bank pairs per 32 lanes. Linear
// because every offset constant is a multiple of 16, or (stride-1 first
// stage) the base is a multiple of R0 = 16 and r < 32 adds whole 16-blocks.
struct RowIdx
{
    __device__ __forceinline__ int base(int b) const { return b + (b >> 4); }
    static constexpr int off(int c) { return c + (c >> 4); }
};

// Columns: element e of column c at e * B + c.
template<int B>
struct ColIdx
{
    int c;
    __device__ __forceinline__ int base(int b) const { return b * B + c; }
    static constexpr int off(int e) { return e * B; }
};

// Opaque copy: stops the compiler hoisting per-element addresses (one
// register each) out of the row / column-block loops.
__device__ __forceinline__ int opaque(int x)
{
    asm volatile("" : "+v"(x));
    return x;
}

// Raw buffer view of float2 data: one 32-bit per-thread byte offset
// (voffset) plus a wave-uniform byte offset (soffset, scalar register), so a
// thread's EPT loads / stores share a single address register.
struct Buf
{
    __amdgpu_buffer_rsrc_t rsrc;

    __device__ __forceinline__ Buf(const void* base, uint32_t bytes)
    {
        rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                (int)bytes, 0x00020000);
    }

    __device__ __forceinline__ float2 load(uint32_t voff, uint32_t soff) const
    {
        return __builtin_bit_cast(float2,
                __builtin_amdgcn_raw_buffer_load_b64(rsrc, voff, soff, 0));
    }

    __device__ __forceinline__ void store(float2 x, uint32_t voff,
            uint32_t soff) const
    {
        using V = decltype(__builtin_amdgcn_raw_buffer_load_b64(rsrc, 0, 0, 0));
        __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(V, x), rsrc,
                voff, soff, 0);
    }

    // Predicated forms without branches: a disabled lane addresses past
    // num_records, so the hardware range check returns 0 / drops the store
    // (a branch per element would make the compiler wait for each load).
    __device__ __forceinline__ float2 load_if(bool ok, uint32_t voff) const
    {
        return load(ok ? voff : kOutOfRange, 0);
    }

    __device__ __forceinline__ void store_if(bool ok, float2 x,
            uint32_t voff) const
    {
        store(x, ok ? voff : kOutOfRange, 0);
    }

    static constexpr uint32_t kOutOfRange = 0xFFFFFFF0u;
};

// Same for 32-bit floats (the image).
struct BufF
{
    __amdgpu_buffer_rsrc_t rsrc;

    __device__ __forceinline__ BufF(const void* base, uint32_t bytes)
    {
        rsrc = __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0,
                (int)bytes, 0x00020000);
    }

    __device__ __forceinline__ float load_if(bool ok, uint32_t voff) const
    {
        return __builtin_bit_cast(float, __builtin_amdgcn_raw_buffer_load_b32(
                rsrc, ok ? voff : Buf::kOutOfRange, 0, 0));
    }

    __device__ __forceinline__ void store_if(bool ok, float x,
            uint32_t voff) const
    {
        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(
                decltype(__builtin_amdgcn_raw_buffer_load_b32(rsrc, 0, 0, 0)),
                x), rsrc, ok ? voff : Buf::kOutOfRange, 0, 0);
    }
};

// Gridding ------------------------------------------------------------------
//
// Buffer views of the grid: byte offset = uniform part (row / column-block
// constants, SGPR) + per-thread part (p and the column, one VGPR). Row
// passes view the grid from k0 cells before its start so that the cropped
// column e - k0 of a row is at offset row * G + e (never negative).

constexpr uint32_t grid_bytes(int G, int k0)
{
    return (uint32_t)(((size_t)G * G + k0) * sizeof(float2));
}

// Row pass (inverse): grid row u -> its M centre outputs, in place.
template<int G>
__global__ void __launch_bounds__(RowPlan<G>::P)
k_rows_grid(float2* __restrict__ grid, int k0, int M,
        const float2* __restrict__ W, const uint32_t* __restrict__ tiles,
        int ncoarse)
{
    using F = RowFft<G, 1>;
    static_assert(F::EPT <= 32, "one mask bit per element");
    extern __shared__ float2 lds[];
    const int p = threadIdx.x;
    const Buf gb(grid - k0, grid_bytes(G, k0));
    F f;
    f.init(p, W, G);
    // Contiguous blocks of rows per workgroup (whole 64-row tile rows for
    // the usual G / gridDim): the thread's element mask of occupied tiles
    // is rebuilt only when the tile row changes. Element c of a thread
    // (column p + c, c a multiple of P) is bit c / P.
    const int per = (G + gridDim.x - 1) / gridDim.x;
    const int r_begin = blockIdx.x * per, r_end = min(G, r_begin + per);
    uint32_t occ = ~0u;
    int occ_row = -1;
    for (int row = r_begin; row < r_end; ++row)
    {
        const int pq = opaque(p);
        if (tiles && (row >> 6) != occ_row)
        {
            // Tiles with no bucketed visibility were not written by the
            // scatter (their cells are zero): read nothing for them.
            occ_row = row >> 6;
            occ = 0u;
#pragma unroll
            for (int b = 0; b < F::EPT; ++b)
            {
                const unsigned tu = (unsigned)occ_row;
                const unsigned tv = (unsigned)(pq + b * RowPlan<G>::P) >> 6;
                const unsigned bin = (((tu >> 2) * (unsigned)ncoarse +
                        (tv >> 2)) << 4) | ((tu & 3u) << 2) | (tv & 3u);
                if (tiles[bin] != 0u) occ |= 1u << b;
            }
        }
        const uint32_t vo = (uint32_t)pq * 8u;
        const uint32_t ro = ((uint32_t)row * G + k0) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int c) {
            return gb.load_if((occ >> (c / RowPlan<G>::P)) & 1u,
                    vo + ro + c * 8u);
        });
        f.transform(v, pq, lds, RowIdx{});
        const uint32_t vr = (uint32_t)row * G * 8u + vo;
        F::store_output(v, [&](int c, int, float2 x) {
            gb.store_if((unsigned)(pq + c - k0) < (unsigned)M, x, vr + c * 8u);
        });
    }
}

// Column pass A (inverse): for u1 = blockIdx.x, length-N2 FFTs over rows
// u1 + N1 * n2, times W^(u1 k2)*, back into rows u1 + N1 * k2.
template<int N1, int N2, int SIGN = 1>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDP_COLA_WAVES)))
k_cols_a_grid(float2* __restrict__ grid, int M, const float2* __restrict__ W)
{
    constexpr int G = N1 * N2, B = ColPlan<N2>::B;
    using F = ColFft<N2, SIGN>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int u1 = blockIdx.x;
    const Buf gb(grid, grid_bytes(G, 0));
    F f;
    f.init(p, W, G);
    float2 fs[F::EPT];
#pragma unroll
    for (int i = 0; i < F::EPT; ++i)
        fs[i] = F::twiddle(W, u1 * F::out_index(p, i));
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)u1 * G * 8u;
    constexpr uint32_t kStep = (uint32_t)N1 * G * 8u;   // one n2 / k2 step
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const bool ok = col < M;
        const uint32_t vo = ((uint32_t)pq * N1 * G + col) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int e) {
            return ok ? gb.load(vo, so + e * kStep) : make_float2(0.f, 0.f);
        });
        f.transform(v, pq, lds, ColIdx<B>{cq});
        F::store_output(v, [&](int e, int i, float2 x) {
            if (ok) gb.store(cmul(x, fs[i]), vo, so + e * kStep);
        });
    }
}

// Column pass B (inverse) + image epilogue: for k2 = blockIdx.x, length-N1
// FFTs over rows N1 * k2 + n1; output row k = k2 + N2 * k1 is image row
// k - k0. 2-D: dirty = (dirty + checker * Re) / correction
// (conv_corr_and_scaling, sdp_gridder_uvw_es_fft.cpp:706-740); 3-D:
// dirty += checker * Re(F * phasor(w)) (apply_w_screen_and_sum, :664-700).
template<int N1, int N2, bool DO_W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDP_COLB_WAVES)))
k_cols_b_grid(const float2* __restrict__ grid, float* __restrict__ dirty,
        ImageParams<float> ip, int plane, int k0, int M,
        const float2* __restrict__ W)
{
#pragma clang fp contract(off)
    constexpr int G = N1 * N2, B = ColPlan<N1>::B;
    using F = ColFft<N1, 1>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int k2 = blockIdx.x;
    const int h = M / 2;
    const Buf gb(grid, grid_bytes(G, 0));
    const BufF db(dirty, (uint32_t)((size_t)ip.N * ip.N * 4));
    F f;
    f.init(p, W, G);
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)N1 * k2 * G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const bool ok = col < M;
        const uint32_t vo = ((uint32_t)pq * G + col) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int e) {
            return ok ? gb.load(vo, so + e * (uint32_t)G * 8u)
                      : make_float2(0.f, 0.f);
        });
        // The image values this thread adds to, loaded ahead of the
        // transform: a load between two stores to the same image would
        // wait for the store before it (possible alias), one round trip
        // per element.
        float prev[F::EPT];
#pragma unroll
        for (int i = 0; i < F::EPT; ++i)
        {
            const int iy = k2 + N2 * F::out_index(pq, i) - k0;
            const bool in = ok && (unsigned)iy < (unsigned)M;
            prev[i] = db.load_if(in, ((uint32_t)iy * ip.N + col) * 4u);
        }
        f.transform(v, pq, lds, ColIdx<B>{cq});
        const float ccx = ip.conv_corr[min(abs(col - h), h)];
        F::store_output(v, [&](int e, int i, float2 x) {
            const int iy = k2 + N2 * (pq + e) - k0;
            const bool in = ok && (unsigned)iy < (unsigned)M;
            const int ix = col;
            const int xo = ix - h, yo = iy - h;
            const uint32_t off = ((uint32_t)iy * ip.N + ix) * 4u;
            float val;
            if constexpr (DO_W)
            {
                // Only the image rows need the w-screen (a third of the
                // padded rows are cropped; rows are wave-uniform).
                float re = 0.0f, im = 0.0f;
                if (in) phasor(ip, plane, abs(xo), abs(yo), -1.0f, re, im);
                val = x.x * re - x.y * im;
            }
            else
            {
                val = x.x;
            }
            if ((ix + iy) & 1) val = -val;
            float out = prev[i] + val;
            if constexpr (!DO_W)
            {
                // inv_correction (es_image_dev.h), 2-D branch, same order.
                const float ccy = ip.conv_corr[min(abs(yo), h)];
                const float corr = ccx * ccy * ip.norm * ip.norm;
                out *= 1.0f / corr;
            }
            db.store_if(in, out, off);
        });
    }
}

// Gridding, 2-D: the real-output form ---------------------------------------
//
// The 2-D gridder keeps only Re of the transform (checkerboard and
// correction are real), and Re(IDFT2(A)) = IDFT2(H) with the Hermitian part
// H[u][v] = (A[u][v] + conj(A[-u][-v])) / 2 (indices mod G). The row
// transforms Bh[u][x] of H are Hermitian down every column (Bh[-u][x] =
// conj(Bh[u][x])), so the column transform is complex-to-real: with
// Xe[k] = Bh[k] + conj(Bh[G/2 - k]) and Xo[k] = (Bh[k] - conj(Bh[G/2 - k]))
// e^{2 pi i k / G}, the length-G/2 transform z of Z = Xe + i Xo gives the
// output rows 2m (Re z[m]) and 2m + 1 (Im z[m]). The row pass forms Z
// directly: one workgroup per quad of grid rows {k, G - k, G/2 - k,
// G/2 + k} (k = 0: {0, G/2}; k = G/4: {G/4, 3G/4}; the quads partition the
// rows, so the pass stays in place) transforms the H rows k and G/2 - k and
// writes the Z rows k and G/2 - k. The column passes then move G/2 rows
// instead of G and the row pass writes half as much: ~1.3 GB of HBM
// traffic per call at config 2 instead of ~2.0 GB, and half the column
// FFT work.

// Split of the half-length column transform, G2 = N1 * N2. At G2 = 4096
// (config 2) 32 x 128 beat 64 x 64 and 128 x 32 (A/B: gridding FFT 0.288
// -> 0.259 ms, degridding image pass 0.113 -> 0.090 ms): the strided pass
// then runs 128-point columns over rows 32 apart.
template<int G2> struct HalfSplit;
template<> struct HalfSplit<1024> { static constexpr int N1 = 32, N2 = 32; };
template<> struct HalfSplit<2048> { static constexpr int N1 = 32, N2 = 64; };
template<> struct HalfSplit<4096> { static constexpr int N1 = 32, N2 = 128; };

// Occupancy of the row pass's loads. With P = G / 16 threads per row and
// 16 elements each, thread p's element r of a row sits at column p + r P
// (tile p / 64 + r S, S = P / 64) and its partner element at column
// (G - p - r P) mod G (tile (T - ceil(p / 64) - r S) mod T, T = G / 64
// tiles per row). So per tile row and thread class one 32-bit word holds
// the 16 bits of both: low half forward (class p / 64), high half reversed
// (class ceil(p / 64)), S + 1 classes.
__host__ __device__ constexpr int occ_classes(int G)
{
    return G / 1024 + 1;
}

// One block per tile row, one thread per bit: thread t builds bit t % 32
// of class t / 32's word (bits 0-15 forward, 16-31 reversed), and a wave's
// ballot holds the words of two classes.
// HALO (degridding): a tile counts if it or its upper / left / upper-left
// neighbour holds entries (the gather's reach, as k_rows_image).
template<bool HALO>
__global__ void __launch_bounds__(320) k_row_occupancy(
        const uint32_t* __restrict__ tiles, int ncoarse, int G,
        uint32_t* __restrict__ occ)
{
    const int T = G / 64, S = G / 1024;
    const int t = threadIdx.x, cls = t >> 5, j = t & 31, r = j & 15;
    const unsigned tu = blockIdx.x;
    int tv = -1;
    if (cls <= S)
    {
        if (j < 16) tv = cls < S ? cls + r * S : -1;
        else tv = ((T - cls - r * S) % T + T) % T;
    }
    auto count = [&](int a, int b) -> uint32_t {
        if (a < 0 || b < 0) return 0u;
        const unsigned x = (unsigned)a, y = (unsigned)b;
        return tiles[(((x >> 2) * (unsigned)ncoarse + (y >> 2)) << 4) |
                ((x & 3u) << 2) | (y & 3u)];
    };
    bool bit = false;
    if (tv >= 0)
    {
        const int a = (int)tu;
        bit = HALO ? (count(a, tv) | count(a - 1, tv) | count(a, tv - 1) |
                count(a - 1, tv - 1)) != 0u : count(a, tv) != 0u;
    }
    const uint64_t m = __ballot(bit);
    if (j == 0 && cls <= S)
        occ[tu * (S + 1) + cls] = (uint32_t)(m >> (t & 32));
}

// Single-row form of the real-output row pass: one
// H row per iteration, H[u] = (A[u] + conj A[-u](-v)) / 2 for u = 0 .. G/2,
// transformed and written as Bh[u] (M centre columns) into grid row u. A
// workgroup is one row's threads and LDS (RowPlan<G>), so two share a CU and
// one's loads overlap the other's transform (the quad form holds both rows
// of a pair in one 1024-thread workgroup, one per CU). Grid rows u and G - u
// are read only by row u's iteration, so the pass stays in place. The pair
// mixing Z = Xe + i Xo moves into the first column pass
// (k_cols_a_herm_pairs).
template<int G>
__global__ void __launch_bounds__(RowPlan<G>::P)
k_rows_herm1(float2* __restrict__ grid, int k0, int M,
        const float2* __restrict__ W, const uint32_t* __restrict__ occ)
{
    using F = RowFft<G, 1>;
    constexpr int P = RowPlan<G>::P, EPT = F::EPT;
    constexpr int NC = occ_classes(G), NH = G / 2 + 1;
    static_assert(EPT == 16 && P == G / 16 && P % 64 == 0,
            "element r of thread p at column p + r P (k_row_occupancy)");
    extern __shared__ float2 lds[];
    const int p = threadIdx.x;
    const Buf gb(grid - k0, grid_bytes(G, k0));
    F f;
    f.init(p, W, G);
    const int per = (NH + gridDim.x - 1) / gridDim.x;
    const int u_begin = blockIdx.x * per, u_end = min(NH, u_begin + per);
    for (int u = u_begin; u < u_end; ++u)
    {
        const int pq = opaque(p);
        const int ur = (G - u) & (G - 1);
        const uint32_t oa_bits = occ ?
                occ[(u >> 6) * NC + (pq >> 6)] : 0xFFFFFFFFu;
        const uint32_t ob_bits = occ ?
                occ[(ur >> 6) * NC + ((pq + 63) >> 6)] >> 16 : 0xFFFFFFFFu;
        const uint32_t ra = ((uint32_t)u * G + k0) * 8u;
        const uint32_t rb = ((uint32_t)ur * G + k0) * 8u;
        float2 v[EPT];
        F::load_input(v, [&](int c) {
            const int ca = pq + c, cb = (G - ca) & (G - 1);
            const bool oa = (oa_bits >> (c / P)) & 1u;
            const bool ob = (ob_bits >> (c / P)) & 1u;
            const float2 a = gb.load_if(oa, ra + (uint32_t)ca * 8u);
            const float2 b = gb.load_if(ob, rb + (uint32_t)cb * 8u);
            return make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
        });
        f.transform(v, pq, lds, RowIdx{});
        const uint32_t vr = (uint32_t)u * G * 8u + (uint32_t)pq * 8u;
        F::store_output(v, [&](int c, int, float2 x) {
            gb.store_if((unsigned)(pq + c - k0) < (unsigned)M, x, vr + c * 8u);
        });
    }
}

// Column pass A of the half-length transform on the Bh rows of
// k_rows_herm1: it first forms the Z rows, Z[m] = (Bh[m] + conj Bh[G/2 - m])
// + i (Bh[m] - conj Bh[G/2 - m]) e^{2 pi i m / G}, then runs k_cols_a_herm's
// length-N2 transforms. Rows m = u1 + N1 n2 (class u1) pair with element
// N2 - 1 - n2 of class N1 - u1, so workgroup j takes the classes j and
// N1 - j. Thread p holds elements n2 = p + PT r of class j and, loaded as
// thread p' = PT - 1 - p would, the mirrored elements N2 - 1 - n2 of class
// N1 - j: every pair meets in one thread's registers (no exchange), and
// the thread then transforms class N1 - j in the role of thread p' (slot
// 15 - r). Workgroup 0 (class 0: element n2 pairs with N2 - n2, element 0
// with Bh[G/2]) and workgroup N1/2 (class N1/2 with itself) load their
// partners a second time and transform one class.
// Two waves per SIMD (3 measured 118 vs 110 us). 256 threads per
// workgroup = 32 columns of 8 threads (256-byte row segments); 512 (64
// columns, 512-byte segments) measured 110.9 -> 112.4 us.
#define SDP_PAIRS_WAVES 2
constexpr int kPairsThreads = 256;
template<int N1, int N2, int NTH = kPairsThreads>
__global__ void __launch_bounds__(NTH) __attribute__((amdgpu_waves_per_eu(SDP_PAIRS_WAVES)))
k_cols_a_herm_pairs(float2* __restrict__ grid, int M,
        const float2* __restrict__ W)
{
    constexpr int PT = ColPlan<N2>::P, B = NTH / PT;
    constexpr int G = 2 * N1 * N2;
    using F = ColFft<N2, 1>;
    static_assert(F::EPT == 16 && PT * 16 == N2, "element n2 = p + PT r");
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int ja = blockIdx.x, jb = N1 - ja;      // ja = 0: jb unused
    const bool pair = ja != 0 && 2 * ja != N1;
    const Buf gb(grid, grid_bytes(G, 0));
    F f;
    const int ncb = (M + B - 1) / B;
    constexpr uint32_t kStep = (uint32_t)N1 * G * 8u;   // one n2 / k2 step
    const uint32_t so_a = (uint32_t)ja * G * 8u;
    const uint32_t so_b = (uint32_t)(jb & (N1 - 1)) * G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int pm = PT - 1 - pq;                   // mirror thread
        const int col = cb * B + cq;
        const bool ok = col < M;
        float2 za[16], zb[16];
        // Own elements of class ja; partners: class 0 element N2 - n2
        // (row N1 (N2 - n2); n2 = 0 -> row G/2), else element N2 - 1 - n2
        // of class jb (class ja itself for ja = N1/2).
#pragma unroll
        for (int r = 0; r < 16; ++r)
        {
            const int n2 = pq + PT * r;
            const uint32_t co = (uint32_t)col * 8u;
            za[r] = ok ? gb.load(co + (uint32_t)n2 * kStep, so_a)
                       : make_float2(0.f, 0.f);
            const int n2p = ja == 0 ? N2 - n2 : N2 - 1 - n2;
            zb[r] = ok ? gb.load(co + (uint32_t)n2p * kStep,
                    ja == 0 ? 0u : so_b) : make_float2(0.f, 0.f);
        }
#pragma unroll
        for (int r = 0; r < 16; ++r)
        {
            const int n2 = pq + PT * r;
            const int n2p = ja == 0 ? N2 - n2 : N2 - 1 - n2;
            const float2 a = za[r], b = zb[r];
            const float2 wa = W[ja + N1 * n2];            // conj: e^{+}
            const float2 xa = make_float2(a.x + b.x, a.y - b.y);
            const float2 ya = cmul(make_float2(a.x - b.x, a.y + b.y),
                    make_float2(wa.x, -wa.y));
            za[r] = make_float2(xa.x - ya.y, xa.y + ya.x);
            if (pair)
            {
                const float2 wb = W[jb + N1 * n2p];
                const float2 xb = make_float2(b.x + a.x, b.y - a.y);
                const float2 yb = cmul(make_float2(b.x - a.x, b.y + a.y),
                        make_float2(wb.x, -wb.y));
                zb[r] = make_float2(xb.x - yb.y, xb.y + yb.x);
            }
        }
        f.init(pq, W, G);
        f.transform(za, pq, lds, ColIdx<B>{cq});
        const uint32_t vo = ((uint32_t)pq * N1 * G + col) * 8u;
        F::store_output(za, [&](int e, int i, float2 x) {
            const float2 fs = F::twiddle(W, 2 * ja * F::out_index(pq, i));
            if (ok) gb.store(cmul(x, fs), vo, so_a + e * kStep);
        });
        if (pair)
        {
            // Class jb in the role of the mirror thread: its slot r' holds
            // element pm + PT r', i.e. this thread's slot 15 - r'.
            float2 v[16];
#pragma unroll
            for (int r = 0; r < 16; ++r) v[r] = zb[15 - r];
            f.init(pm, W, G);
            f.transform(v, pm, lds, ColIdx<B>{cq});
            const uint32_t vb = ((uint32_t)pm * N1 * G + col) * 8u;
            F::store_output(v, [&](int e, int i, float2 x) {
                const float2 fs = F::twiddle(W, 2 * jb * F::out_index(pm, i));
                if (ok) gb.store(cmul(x, fs), vb, so_b + e * kStep);
            });
        }
    }
}

// Column pass B of the half-length transform + 2-D image epilogue: for
// k2 = blockIdx.x, length-N1 FFTs over rows N1 * k2 + n1; z[m], m = k2 +
// N2 * k1, is Re: output row 2m, Im: output row 2m + 1 (image rows minus
// k0), each then as k_cols_b_grid: dirty = (dirty + checker * f) /
// correction.
template<int N1, int N2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDP_COLB_WAVES)))
k_cols_b_herm(const float2* __restrict__ grid, float* __restrict__ dirty,
        ImageParams<float> ip, int k0, int M, const float2* __restrict__ W)
{
#pragma clang fp contract(off)
    constexpr int G = 2 * N1 * N2, B = ColPlan<N1>::B;
    using F = ColFft<N1, 1>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int k2 = blockIdx.x;
    const int h = M / 2;
    const Buf gb(grid, grid_bytes(G, 0));
    const BufF db(dirty, (uint32_t)((size_t)ip.N * ip.N * 4));
    F f;
    f.init(p, W, G);
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)N1 * k2 * G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const bool ok = col < M;
        const uint32_t vo = ((uint32_t)pq * G + col) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int e) {
            return ok ? gb.load(vo, so + e * (uint32_t)G * 8u)
                      : make_float2(0.f, 0.f);
        });
        // The image values this thread adds to, loaded ahead of the
        // transform (see k_cols_b_grid).
        float prev[F::EPT][2];
#pragma unroll
        for (int i = 0; i < F::EPT; ++i)
#pragma unroll
            for (int j = 0; j < 2; ++j)
            {
                const int iy = 2 * (k2 + N2 * F::out_index(pq, i)) + j - k0;
                const bool in = ok && (unsigned)iy < (unsigned)M;
                prev[i][j] = db.load_if(in, ((uint32_t)iy * ip.N + col) * 4u);
            }
        f.transform(v, pq, lds, ColIdx<B>{cq});
        const float ccx = ip.conv_corr[min(abs(col - h), h)];
        F::store_output(v, [&](int e, int i, float2 x) {
#pragma unroll
            for (int j = 0; j < 2; ++j)
            {
                const int iy = 2 * (k2 + N2 * (pq + e)) + j - k0;
                const bool in = ok && (unsigned)iy < (unsigned)M;
                const int ix = col;
                const int yo = iy - h;
                const uint32_t off = ((uint32_t)iy * ip.N + ix) * 4u;
                float val = j ? x.y : x.x;
                if ((ix + iy) & 1) val = -val;
                float out = prev[i][j] + val;
                // inv_correction (es_image_dev.h), 2-D branch, same order.
                const float ccy = ip.conv_corr[min(abs(yo), h)];
                const float corr = ccx * ccy * ip.norm * ip.norm;
                out *= 1.0f / corr;
                db.store_if(in, out, off);
            }
        });
    }
}

// Column pass B in place (full 2-D FFTs of a whole grid, w-stacking): for
// k2 = blockIdx.x, length-N1 FFTs over the contiguous rows N1 * k2 + n1,
// output k1 back into row N1 * k2 + k1. Natural row k = k2 + N2 * k1 of the
// transform is then stored at row N1 * (k % N2) + k / N2 (fft_perm_row).
template<int N1, int N2, int SIGN>
__global__ void __launch_bounds__(256)
k_cols_b_block(float2* __restrict__ grid, int M, const float2* __restrict__ W)
{
    constexpr int G = N1 * N2, B = ColPlan<N1>::B;
    using F = ColFft<N1, SIGN>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int k2 = blockIdx.x;
    const Buf gb(grid, grid_bytes(G, 0));
    F f;
    f.init(p, W, G);
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)N1 * k2 * G * 8u;
    constexpr uint32_t kStep = (uint32_t)G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const bool ok = col < M;
        const uint32_t vo = ((uint32_t)pq * G + col) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int e) {
            return ok ? gb.load(vo, so + e * kStep) : make_float2(0.f, 0.f);
        });
        f.transform(v, pq, lds, ColIdx<B>{cq});
        F::store_output(v, [&](int e, int, float2 x) {
            if (ok) gb.store(x, vo, so + e * kStep);
        });
    }
}

// Degridding ----------------------------------------------------------------

// Column pass A (forward) with the image prologue: for n1 = blockIdx.x,
// rows n1 + N1 * n2 of the zero-padded image, length-N2 FFTs, times
// W^(n1 k2), into buffer rows k2 + N2 * n1. Prologue (reverse screen,
// sdp_gridder_uvw_es_fft.cpp:790-880): 2-D corrects the image in place and
// applies the checker; 3-D applies checker * phasor(w).
template<int N1, int N2, bool DO_W>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDP_COLA_WAVES)))
k_cols_a_image(float* __restrict__ dirty, int correct_in_place,
        float2* __restrict__ grid, ImageParams<float> ip, int plane, int k0,
        int M, const float2* __restrict__ W)
{
#pragma clang fp contract(off)
    constexpr int G = N1 * N2, B = ColPlan<N2>::B;
    using F = ColFft<N2, -1>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int n1 = blockIdx.x;
    const int h = M / 2;
    const Buf gb(grid, grid_bytes(G, 0));
    const BufF db(dirty, (uint32_t)((size_t)ip.N * ip.N * 4));
    F f;
    f.init(p, W, G);
    float2 fs[F::EPT];
#pragma unroll
    for (int i = 0; i < F::EPT; ++i)
        fs[i] = F::twiddle(W, n1 * F::out_index(p, i));
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)N2 * n1 * G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const bool ok = col < M;
        float2 v[F::EPT];
        const float ccx = ip.conv_corr[min(abs(col - h), h)];
        // All of the thread's image loads first, then the in-place
        // correction stores: a load behind a store to the same image waits
        // for it (possible alias), one round trip per element.
        static_assert(F::EPT == 16, "one input slot per element (R0 = 16)");
        F::load_input(v, [&](int e) {
            const int iy = n1 + N1 * (pq + e) - k0;
            const bool in = ok && (unsigned)iy < (unsigned)M;
            return make_float2(db.load_if(in,
                    ((uint32_t)iy * ip.N + col) * 4u), 0.0f);
        });
        F::load_input(v, [&](int e) {
            const int iy = n1 + N1 * (pq + e) - k0;
            const bool in = ok && (unsigned)iy < (unsigned)M;
            const int ix = col;
            const int xo = ix - h, yo = iy - h;
            const uint32_t off = ((uint32_t)iy * ip.N + ix) * 4u;
            float val = v[e / (N2 / 16)].x;
            if constexpr (!DO_W)
            {
                // The 3-D path corrects the whole image before the planes.
                if (correct_in_place)
                {
                    // inv_correction (es_image_dev.h), 2-D branch.
                    const float ccy = ip.conv_corr[min(abs(yo), h)];
                    const float corr = ccx * ccy * ip.norm * ip.norm;
                    val *= 1.0f / corr;
                    db.store_if(in, val, off);
                }
            }
            if ((ix + iy) & 1) val = -val;
            float pr = 1.0f, pi = 0.0f;
            // The zero-padding rows (val = 0) need no w-screen.
            if constexpr (DO_W)
                if (in) phasor(ip, plane, abs(xo), abs(yo), 1.0f, pr, pi);
            return make_float2(pr * val, pi * val);
        });
        f.transform(v, pq, lds, ColIdx<B>{cq});
        const uint32_t vo = ((uint32_t)pq * G + col) * 8u;
        F::store_output(v, [&](int e, int i, float2 x) {
            if (ok) gb.store(cmul(x, fs[i]), vo, so + e * (uint32_t)G * 8u);
        });
    }
}

// Column pass B (forward): for k2 = blockIdx.x, length-N1 FFTs over rows
// k2 + N2 * n1, results back into rows k2 + N2 * k1 (the same rows).
template<int N1, int N2>
__global__ void __launch_bounds__(256)
k_cols_b_image(float2* __restrict__ grid, int M, const float2* __restrict__ W)
{
    constexpr int G = N1 * N2, B = ColPlan<N1>::B;
    using F = ColFft<N1, -1>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int k2 = blockIdx.x;
    const Buf gb(grid, grid_bytes(G, 0));
    F f;
    f.init(p, W, G);
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)k2 * G * 8u;
    constexpr uint32_t kStep = (uint32_t)N2 * G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const bool ok = col < M;
        const uint32_t vo = ((uint32_t)pq * N2 * G + col) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int e) {
            return ok ? gb.load(vo, so + e * kStep) : make_float2(0.f, 0.f);
        });
        f.transform(v, pq, lds, ColIdx<B>{cq});
        F::store_output(v, [&](int e, int, float2 x) {
            if (ok) gb.store(x, vo, so + e * kStep);
        });
    }
}

// Row pass (forward): row k holds its M centre inputs at [0, M); zero-pad,
// transform, write all G cells of the row.
template<int G>
__global__ void __launch_bounds__(RowPlan<G>::P)
k_rows_image(float2* __restrict__ grid, int k0, int M,
        const float2* __restrict__ W, const uint32_t* __restrict__ tiles,
        int ncoarse)
{
    using F = RowFft<G, -1>;
    constexpr int P = RowPlan<G>::P;
    static_assert(F::EPT <= 32, "one mask bit per element");
    extern __shared__ float2 lds[];
    const int p = threadIdx.x;
    const Buf gb(grid - k0, grid_bytes(G, k0));
    F f;
    f.init(p, W, G);
    // As k_rows_grid: contiguous row blocks and a per-thread element mask,
    // here of the tiles the gather will read -- tile (tu, tv) is read by
    // the visibilities bucketed in it and (halo, taps reach <= 16 cells
    // past a tile) in the tiles above and to the left of it.
    const int per = (G + gridDim.x - 1) / gridDim.x;
    const int r_begin = blockIdx.x * per, r_end = min(G, r_begin + per);
    const int nt = G / kTile;
    auto count = [&](int tu, int tv) -> uint32_t {
        if (tu < 0 || tv < 0) return 0u;
        const unsigned u = (unsigned)tu, v = (unsigned)tv;
        return tiles[(((u >> 2) * (unsigned)ncoarse + (v >> 2)) << 4) |
                ((u & 3u) << 2) | (v & 3u)];
    };
    uint32_t need = ~0u;
    int need_row = -1;
    for (int row = r_begin; row < r_end; ++row)
    {
        const int pq = opaque(p);
        if (tiles && (row >> 6) != need_row)
        {
            need_row = row >> 6;
            need = 0u;
#pragma unroll
            for (int b = 0; b < F::EPT; ++b)
            {
                const int tu = need_row, tv = (pq + b * P) >> 6;
                if (tv < nt && (count(tu, tv) | count(tu - 1, tv) |
                        count(tu, tv - 1) | count(tu - 1, tv - 1)))
                    need |= 1u << b;
            }
        }
        const uint32_t vo = (uint32_t)pq * 8u;
        const uint32_t rs = (uint32_t)row * G * 8u;
        float2 v[F::EPT];
        const uint32_t vr = rs + vo;
        F::load_input(v, [&](int c) {
            return gb.load_if((unsigned)(pq + c - k0) < (unsigned)M,
                    vr + c * 8u);
        });
        f.transform(v, pq, lds, RowIdx{});
        const uint32_t ro = ((uint32_t)row * G + k0) * 8u;
        F::store_output(v, [&](int c, int, float2 x) {
            // Output element c of the thread is column p + c (c / P its
            // mask bit); tiles nobody reads are not written.
            gb.store_if((need >> (c / P)) & 1u, x, vo + ro + c * 8u);
        });
    }
}

// Degridding, 2-D: the real-input form -------------------------------------
//
// The corrected image is real, so its transform is Hermitian: A[-u][-v] =
// conj(A[u][v]). The column passes transform the image row pairs
// z[m] = f[2m] + i f[2m + 1] with a length-G/2 complex transform Z
// (four-step over G/2 rows of the grid buffer), and the row pass recovers
// the column spectra X[k] = (Z[k] + conj Z[G/2 - k]) / 2 - i (Z[k] -
// conj Z[G/2 - k]) e^{-2 pi i k / G} / 2, k in [0, G/2], from quads (Z rows
// k and G/2 - k, swapped between the two halves of the workgroup through
// LDS), transforms them along the rows and writes each grid row u together
// with row G - u, the conjugate of row u reversed. Traffic per call at
// config 2: ~1.3 GB instead of ~2.1 GB.

// Column pass A (forward) with the 2-D image prologue: for n1 = blockIdx.x,
// length-N2 FFTs over m = n1 + N1 n2 of z[m] = f[2m] + i f[2m + 1] (image
// rows 2m - k0 and 2m + 1 - k0, corrected in place, checkerboard), times
// e^{-2 pi i n1 k2 / (G/2)}, into rows N2 n1 + k2 (row pitch G).
template<int N1, int N2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(3)))
k_cols_a_image_herm(float* __restrict__ dirty, float2* __restrict__ grid,
        ImageParams<float> ip, int k0, int M, const float2* __restrict__ W)
{
#pragma clang fp contract(off)
    constexpr int G = 2 * N1 * N2, B = ColPlan<N2>::B;
    using F = ColFft<N2, -1>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int n1 = blockIdx.x;
    const int h = M / 2;
    const Buf gb(grid, grid_bytes(G, 0));
    const BufF db(dirty, (uint32_t)((size_t)ip.N * ip.N * 4));
    F f;
    f.init(p, W, G);
    float2 fs[F::EPT];
#pragma unroll
    for (int i = 0; i < F::EPT; ++i)
        fs[i] = F::twiddle(W, 2 * n1 * F::out_index(p, i));
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)N2 * n1 * G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const bool ok = col < M;
        float2 v[F::EPT];
        const float ccx = ip.conv_corr[min(abs(col - h), h)];
        // All image loads first, then the in-place correction stores (see
        // k_cols_a_image).
        static_assert(F::EPT == 16, "one input slot per element (R0 = 16)");
        F::load_input(v, [&](int e) {
            const int iy = 2 * (n1 + N1 * (pq + e)) - k0;
            const bool in0 = ok && (unsigned)iy < (unsigned)M;
            const bool in1 = ok && (unsigned)(iy + 1) < (unsigned)M;
            return make_float2(
                    db.load_if(in0, ((uint32_t)iy * ip.N + col) * 4u),
                    db.load_if(in1, ((uint32_t)(iy + 1) * ip.N + col) * 4u));
        });
        F::load_input(v, [&](int e) {
            const int iy0 = 2 * (n1 + N1 * (pq + e)) - k0;
            const float2 x = v[e / (N2 / 16)];
            float out[2];
#pragma unroll
            for (int j = 0; j < 2; ++j)
            {
                const int iy = iy0 + j;
                const bool in = ok && (unsigned)iy < (unsigned)M;
                float val = j ? x.y : x.x;
                // inv_correction (es_image_dev.h), 2-D branch.
                const float ccy = ip.conv_corr[min(abs(iy - h), h)];
                const float corr = ccx * ccy * ip.norm * ip.norm;
                val *= 1.0f / corr;
                db.store_if(in, val, ((uint32_t)iy * ip.N + col) * 4u);
                if ((col + iy) & 1) val = -val;
                out[j] = val;
            }
            return make_float2(out[0], out[1]);
        });
        f.transform(v, pq, lds, ColIdx<B>{cq});
        const uint32_t vo = ((uint32_t)pq * G + col) * 8u;
        F::store_output(v, [&](int e, int i, float2 x) {
            if (ok) gb.store(cmul(x, fs[i]), vo, so + e * (uint32_t)G * 8u);
        });
    }
}

// Column pass B (forward) of the half-length transform in the single-row
// form: after the length-N1 transforms it recovers
// the column spectra X[k] = (Z[k] + conj Z[G/2 - k]) / 2 - i (Z[k] - conj
// Z[G/2 - k]) e^{-2 pi i k / G} / 2 itself and writes X[k] into row k
// (k in [0, G/2]; X[G/2] from Z[0]), so the row pass takes one row per
// workgroup iteration (k_rows_image_herm1). Z rows k = k2 + N2 k1 of class
// k2 pair with element N1 - 1 - k1 of class N2 - k2: workgroup j takes the
// classes j and N2 - j, transforming the second in the role of the mirror
// thread p' = PT - 1 - p, whose output slot 15 - i holds exactly the
// partner of this thread's slot i (out_index(p', 15 - i) = N1 - 1 -
// out_index(p, i)); the pairs meet in registers. Workgroup N2/2 (class
// N2/2 with itself) transforms its class twice; workgroup 0 (class 0,
// element k1 paired with N1 - k1 mod N1) exchanges through LDS.
template<int N1, int N2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDP_PAIRS_WAVES)))
k_cols_b_image_herm_pairs(float2* __restrict__ grid, int M,
        const float2* __restrict__ W)
{
    constexpr int G = 2 * N1 * N2, B = ColPlan<N1>::B, PT = ColPlan<N1>::P;
    using F = ColFft<N1, -1>;
    static_assert(F::EPT == 16 && (size_t)N1 * B * sizeof(float2) <=
            kColLdsBytes, "class-0 exchange fits the transform's LDS");
    static_assert(F::out_const(15) + F::out_const(0) == N1 - PT &&
            F::out_const(14) + F::out_const(1) == N1 - PT &&
            F::out_const(9) + F::out_const(6) == N1 - PT,
            "mirror slot 15 - i holds element N1 - 1 - k1");
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int ja = blockIdx.x, jb = N2 - ja;
    const bool two = ja != 0;                    // second transform
    const bool pair = two && 2 * ja != N2;       // second class stored
    const Buf gb(grid, grid_bytes(G, 0));
    F f;
    const int ncb = (M + B - 1) / B;
    constexpr uint32_t kStep = (uint32_t)N2 * G * 8u;
    const uint32_t so_a = (uint32_t)ja * G * 8u;
    const uint32_t so_b = (uint32_t)(jb & (N2 - 1)) * G * 8u;
    auto mix = [](float2 a, float2 b, float2 w) {
        const float2 dw = cmul(make_float2(a.x - b.x, a.y + b.y), w);
        return make_float2(0.5f * ((a.x + b.x) + dw.y),
                0.5f * ((a.y - b.y) - dw.x));
    };
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int pm = PT - 1 - pq;
        const int col = cb * B + cq;
        const bool ok = col < M;
        const uint32_t vo = ((uint32_t)pq * N2 * G + col) * 8u;
        const uint32_t vm = ((uint32_t)pm * N2 * G + col) * 8u;
        float2 va[16], vb[16];
        F::load_input(va, [&](int e) {
            return ok ? gb.load(vo, so_a + e * kStep) : make_float2(0.f, 0.f);
        });
        if (two)
            F::load_input(vb, [&](int e) {
                return ok ? gb.load(vm, so_b + e * kStep)
                          : make_float2(0.f, 0.f);
            });
        f.init(pq, W, G);
        f.transform(va, pq, lds, ColIdx<B>{cq});
        if (two)
        {
            f.init(pm, W, G);
            f.transform(vb, pm, lds, ColIdx<B>{cq});
        }
        else
        {
            // Class 0: partner of k1 is (N1 - k1) mod N1, through LDS.
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 16; ++i)
                lds[F::out_index(pq, i) * B + cq] = va[i];
            __syncthreads();
#pragma unroll
            for (int i = 0; i < 16; ++i)
                vb[15 - i] = lds[((N1 - F::out_index(pq, i)) & (N1 - 1)) * B +
                        cq];
        }
        const float2 z0 = va[0];                 // Z[0] for pq == 0, ja == 0
        // In place: slot i of va and slot 15 - i of vb are read only here.
#pragma unroll
        for (int i = 0; i < 16; ++i)
        {
            const int k1 = F::out_index(pq, i);
            const float2 a = va[i], b = vb[15 - i];
            va[i] = mix(a, b, W[ja + N2 * k1]);            // e^{-2 pi i k / G}
            if (pair)
                vb[15 - i] = mix(b, a, W[jb + N2 * (N1 - 1 - k1)]);
        }
        F::store_output(va, [&](int e, int, float2 x) {
            if (ok) gb.store(x, vo, so_a + e * kStep);
        });
        if (pair)
            F::store_output(vb, [&](int e, int, float2 x) {
                if (ok) gb.store(x, vm, so_b + e * kStep);
            });
        if (ja == 0 && pq == 0 && ok)
            gb.store(mix(z0, z0, make_float2(-1.0f, 0.0f)),
                    ((uint32_t)(G / 2) * G + col) * 8u, 0);
    }
}

// Row pass (forward) of the real-input form, single-row: X row u (u in
// [0, G/2], from k_cols_b_image_herm_pairs) transformed along the row and
// written as grid row u and row G - u (conjugate, reversed). Row u is read
// only by its own iteration and rows above G/2 by nobody, so in place.
template<int G>
__global__ void __launch_bounds__(RowPlan<G>::P)
k_rows_image_herm1(float2* __restrict__ grid, int k0, int M,
        const float2* __restrict__ W, const uint32_t* __restrict__ need)
{
    using F = RowFft<G, -1>;
    constexpr int P = RowPlan<G>::P, EPT = F::EPT;
    constexpr int NC = occ_classes(G), NH = G / 2 + 1;
    static_assert(EPT == 16 && P == G / 16 && P % 64 == 0,
            "element r of thread p at column p + r P (k_row_occupancy)");
    extern __shared__ float2 lds[];
    const int p = threadIdx.x;
    const Buf gb(grid - k0, grid_bytes(G, k0));
    F f;
    f.init(p, W, G);
    const int per = (NH + gridDim.x - 1) / gridDim.x;
    const int u_begin = blockIdx.x * per, u_end = min(NH, u_begin + per);
    for (int u = u_begin; u < u_end; ++u)
    {
        const int pq = opaque(p);
        float2 v[EPT];
        const uint32_t vx = (uint32_t)u * G * 8u + (uint32_t)pq * 8u;
        F::load_input(v, [&](int c) {
            return gb.load_if((unsigned)(pq + c - k0) < (unsigned)M, vx + c * 8u);
        });
        f.transform(v, pq, lds, RowIdx{});
        const int ur = (G - u) & (G - 1);
        const uint32_t nf = need ? need[(u >> 6) * NC + (pq >> 6)] : ~0u;
        const uint32_t nr = need ?
                need[(ur >> 6) * NC + ((pq + 63) >> 6)] >> 16 : ~0u;
        const uint32_t ro = ((uint32_t)u * G + k0) * 8u + (uint32_t)pq * 8u;
        const uint32_t rr = ((uint32_t)ur * G + k0) * 8u;
        F::store_output(v, [&](int c, int, float2 x) {
            gb.store_if((nf >> (c / P)) & 1u, x, ro + c * 8u);
            const int cr = (G - pq - c) & (G - 1);
            gb.store_if(ur != u && ((nr >> (c / P)) & 1u),
                    make_float2(x.x, -x.y), rr + (uint32_t)cr * 8u);
        });
    }
}

// W-stacking image side (w-towers gridder, sdp_grid_wstack_wtower.hip) -------
//
// Gridding a w-stack plane ends with: gather the FFT'd sub-grids of the
// plane into the G x G grid (k_gather_grid), inverse FFT of the grid
// (rows, then the four-step columns), then image += grid_correct(checker(
// IFFT) / G^2) (k_image_update; ref sdp_grid_wstack_wtower.cpp:686-711).
// The kernel below fuses the image update into the last column pass: the
// grid is then written once less (by that pass) and read once less (by
// the image update), 2 GiB each at G = 16384.

// Column pass B (inverse) with the image update: for k2 = blockIdx.x,
// length-N1 FFTs over rows N1 * k2 + n1; natural output row gu = k2 + N2 k1,
// column gv: image[gu][gv] += correct(checker * x * norm) in the order and
// precision of k_image_update (sdp_grid_wstack_wtower.hip; the correction
// of a float grid, correct_scaled_f32: scale in f32, then the w-stack
// phasor of w_offset).
// IK: the image's element kind (AnyView: 0 f32, 1 f64, 2 c64, 3 c128).
template<int N1, int N2, int IK>
__global__ void __launch_bounds__(256)
k_cols_b_wstack_image(const float2* __restrict__ grid, void* image_ptr,
        float norm, sdp_wt::CorrParams cp, const float2* __restrict__ W)
{
#pragma clang fp contract(off)
    constexpr int G = N1 * N2, B = ColPlan<N1>::B;
    constexpr int kGridKind = 2;                  // complex float grid
    using F = ColFft<N1, 1>;
    using R = typename std::conditional<(IK == 1 || IK == 3), double,
            float>::type;
    constexpr bool kCx = IK >= 2;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int k2 = blockIdx.x;
    const Buf gb(grid, grid_bytes(G, 0));
    R* img = (R*)image_ptr;
    F f;
    f.init(p, W, G);
    const int ncb = G / B;
    const uint32_t so = (uint32_t)N1 * k2 * G * 8u;
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const uint32_t vo = ((uint32_t)pq * G + col) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int e) {
            return gb.load(vo, so + e * (uint32_t)G * 8u);
        });
        // The image value and correction scale of an output are read in the
        // epilogue, not ahead of the transform: holding all 16 across it
        // took the kernel to 181 VGPRs (2 waves per SIMD) and 2.67 ms per
        // 16384^2 plane, against 112 VGPRs and 1.68 ms this way.
        const int pm = col - G / 2;
        R prev_re[F::EPT], prev_im[kCx ? F::EPT : 1];
        float sc[F::EPT];
        auto pre = [&](int i) {
            const int64_t gu = k2 + (int64_t)N2 * F::out_index(pq, i);
            const int64_t idx = gu * G + col;
            prev_re[i] = img[kCx ? 2 * idx : idx];
            if constexpr (kCx) prev_im[i] = img[2 * idx + 1];
            const int pl = (int)(gu - G / 2);
            sc[i] = sdp_wt::corr_inside(pl, pm, cp) ?
                    (float)sdp_wt::corr_scale(pl, pm, kGridKind, cp) : 1.0f;
        };
        f.transform(v, pq, lds, ColIdx<B>{cq});
        F::store_output(v, [&](int e, int i, float2 x) {
            pre(i);
            const int64_t gu = k2 + (int64_t)N2 * (pq + e);
            float re = x.x, im = x.y;
            if ((gu + col) & 1)
            {
                re = -re;
                im = -im;
            }
            re *= norm;
            im *= norm;
            sdp_wt::Cx<double> z = sdp_wt::cx<double>(re, im);
            const int pl = (int)(gu - G / 2);
            if (sdp_wt::corr_inside(pl, pm, cp))
                z = sdp_wt::correct_scaled_f32(z, pl, pm, cp, sc[i]);
            const int64_t idx = gu * G + col;
            if constexpr (kCx)
            {
                img[2 * idx] = (R)((double)prev_re[i] + z.re);
                img[2 * idx + 1] = (R)((double)prev_im[i] + z.im);
            }
            else
            {
                img[idx] = (R)((double)prev_re[i] + z.re);
            }
        });
    }
}

// Degridding a w-stack plane starts with grid = checker(degrid_correct(
// (float)image)) and its forward FFT (k_image_to_grid + rows + four-step
// columns; ref sdp_grid_wstack_wtower.cpp:363-375). A 2-D transform may
// take its axes in either order, so here the columns go first and column
// pass A reads the image itself: the grid is neither written by a prologue
// pass nor re-read by the row pass (2 GiB each at G = 16384). Column pass B
// (k_cols_b_block) and the row pass (k_rows_image over whole rows) follow;
// the result has the stored-row permutation of fft2d_inplace_permuted.
//
// Column pass A (forward) with the image prologue: for u1 = blockIdx.x,
// length-N2 FFTs over rows u1 + N1 * n2 of the prologue's values, in the
// order and precision of k_image_to_grid (the image value rounded to
// float, correct_scaled_f32 with the kind-2 scale, checkerboard), times
// W^(u1 k2), into rows u1 + N1 * k2. IK: the image kind (AnyView).
#ifndef SDP_WSA_WAVES
#define SDP_WSA_WAVES 4
#endif
template<int N1, int N2, int IK>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDP_WSA_WAVES)))
k_cols_a_wstack_image(float2* __restrict__ grid, const void* image_ptr,
        sdp_wt::CorrParams cp, const float2* __restrict__ W)
{
#pragma clang fp contract(off)
    constexpr int G = N1 * N2, B = ColPlan<N2>::B;
    constexpr int kGridKind = 2;                  // complex float grid
    using F = ColFft<N2, -1>;
    using R = typename std::conditional<(IK == 1 || IK == 3), double,
            float>::type;
    constexpr bool kCx = IK >= 2;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int u1 = blockIdx.x;
    const Buf gb(grid, grid_bytes(G, 0));
    const R* img = (const R*)image_ptr;
    F f;
    f.init(p, W, G);
    float2 fs[F::EPT];
#pragma unroll
    for (int i = 0; i < F::EPT; ++i)
        fs[i] = F::twiddle(W, u1 * F::out_index(p, i));
    const int ncb = G / B;
    const uint32_t so = (uint32_t)u1 * G * 8u;
    constexpr uint32_t kStep = (uint32_t)N1 * G * 8u;   // one n2 / k2 step
    for (int cb = blockIdx.y; cb < ncb; cb += gridDim.y)
    {
        const int pq = opaque(p), cq = opaque(c);
        const int col = cb * B + cq;
        const int pm = col - G / 2;
        const uint32_t vo = ((uint32_t)pq * N1 * G + col) * 8u;
        float2 v[F::EPT];
        F::load_input(v, [&](int e) {
            const int gu = u1 + N1 * (pq + e);
            const int64_t idx = (int64_t)gu * G + col;
            const float re = (float)img[kCx ? 2 * idx : idx];
            const float im = kCx ? (float)img[2 * idx + 1] : 0.0f;
            sdp_wt::Cx<double> z = sdp_wt::cx<double>(re, im);
            const int pl = gu - G / 2;
            if (sdp_wt::corr_inside(pl, pm, cp))
                z = sdp_wt::correct_scaled_f32(z, pl, pm, cp,
                        (float)sdp_wt::corr_scale(pl, pm, kGridKind, cp));
            float zr = (float)z.re, zi = (float)z.im;
            if ((gu + col) & 1)
            {
                zr = -zr;
                zi = -zi;
            }
            return make_float2(zr, zi);
        });
        f.transform(v, pq, lds, ColIdx<B>{cq});
        F::store_output(v, [&](int e, int i, float2 x) {
            gb.store(cmul(x, fs[i]), vo, so + e * kStep);
        });
    }
}

// Launch helpers --------------------------------------------------------------

int num_cus()
{
    static int n = 0;
    if (!n)
    {
        int dev = 0;
        if (hipGetDevice(&dev) != hipSuccess ||
                hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount,
                        dev) != hipSuccess || n <= 0)
            n = 256;
    }
    return n;
}

template<auto Kernel>
hipError_t allow_lds(size_t bytes)
{
    static size_t done = 0;
    if (bytes <= done) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute((const void*)Kernel,
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) done = bytes;
    return e;
}

int row_blocks(int G)
{
    const int per_cu = (int)std::max<size_t>(1, (160 * 1024) / row_lds_bytes(G));
    return std::min(G, num_cus() * per_cu);
}

// Column-pass workgroups: rounds x the kernel's resident workgroups per CU.
// A launch that is not a whole number of resident rounds leaves its last
// round partly empty: two rounds (4 per CU for the kernels that hold 3
// (VGPRs) cost config 2 0.03 ms of grid FFT + image and 0.05 ms of degrid
// FFT; the degrid column pass B holds 5 (LDS) and ran 1.2 rounds at 6 per
// CU). The two paired column passes of the real-output form
// (k_cols_a_herm_pairs, k_cols_b_image_herm_pairs: 2 resident per CU) and
// the 3-D column pass B run four rounds: config 2, 110.7 -> 105.0 us and
// 97.6 -> 90.6 us (rounds 1 / 3 / 8: 121.9 / 106.2 / 106.0 and 116.9 /
// 95.4 / 99.6 us; the other column passes measured flat or slower past 2).
constexpr int kColRounds = 2;
constexpr int kPairRounds = 4;

template<auto Kernel>
dim3 col_grid(int fixed, int M, int B, int threads = 256,
        size_t lds = kColLdsBytes, int rounds = 0)
{
    static int occ = 0;
    if (!occ)
    {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, Kernel, threads,
                lds) != hipSuccess || n <= 0)
            n = 3;
        occ = n;
    }
    const int ncb = (M + B - 1) / B;
    const int want = num_cus() * occ * (rounds > 0 ? rounds : kColRounds);
    const int split = std::max(1, std::min(ncb, (want + fixed - 1) / fixed));
    return dim3(fixed, split);
}

struct Geometry
{
    int G, M, k0;
};

Geometry geometry(const ImageParams<float>& ip)
{
    Geometry g;
    g.G = ip.G;
    g.M = 2 * (ip.N / 2);
    g.k0 = ip.G / 2 - ip.N / 2;
    return g;
}

template<int N1, int N2>
int grid_rows(const Geometry& g, const float2* W, float2* grid,
        const uint32_t* tiles, int ncoarse, hipStream_t stream)
{
    constexpr int G = N1 * N2;
    sdp_Error st = SDP_SUCCESS;
    const size_t lds = row_lds_bytes(G);
    SDP_HIP_CHECK((allow_lds<k_rows_grid<G>>(lds)), &st);
    if (st) return st;
    k_rows_grid<G><<<row_blocks(G), RowPlan<G>::P, lds, stream>>>(
            grid, g.k0, g.M, W, tiles, ncoarse);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<int N1, int N2>
int grid_cols_a(const Geometry& g, const float2* W, float2* grid,
        hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    k_cols_a_grid<N1, N2><<<col_grid<k_cols_a_grid<N1, N2>>(N1, g.M,
            ColPlan<N2>::B), 256,
            kColLdsBytes, stream>>>(grid, g.M, W);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<int N1, int N2>
int grid_to_image(const Geometry& g, const ImageParams<float>& ip, int plane,
        const float2* W, const float2* grid, float* dirty, hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    // 3-D (w-stacking) planes: four rounds (config-2 geometry, 10 planes:
    // 167.2 -> 160.5 us per plane; the 2-D form stays on col_rounds()).
    const dim3 blocks = ip.do_w ?
            col_grid<k_cols_b_grid<N1, N2, true>>(N2, g.M, ColPlan<N1>::B,
                    256, kColLdsBytes, kPairRounds) :
            col_grid<k_cols_b_grid<N1, N2, false>>(N2, g.M, ColPlan<N1>::B);
    if (ip.do_w)
        k_cols_b_grid<N1, N2, true><<<blocks, 256, kColLdsBytes, stream>>>(
                grid, dirty, ip, plane, g.k0, g.M, W);
    else
        k_cols_b_grid<N1, N2, false><<<blocks, 256, kColLdsBytes, stream>>>(
                grid, dirty, ip, plane, g.k0, g.M, W);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

// Real-output (Hermitian) form of the 2-D gridding transform, for grids of
// 2048 to 8192 (at 16384 the row pass's rows do not fit the registers; the
// complex form serves 1024 and 16384, and every 3-D plane).
bool herm_enabled(const ImageParams<float>& ip)
{
    return !ip.do_w && ip.G >= 2048 && ip.G <= 8192;
}

// The same for degridding (real-input form).
bool herm_degrid_enabled(const ImageParams<float>& ip)
{
    return !ip.do_w && ip.G >= 2048 && ip.G <= 8192;
}

template<int N1, int N2>
int grid_rows_herm(const Geometry& g, const float2* W, float2* grid,
        const uint32_t* tiles, int ncoarse, uint32_t* occ,
        hipStream_t stream)
{
    constexpr int G = N1 * N2;
    if constexpr (G < 2048 || G > 8192)
    {
        return SDP_ERR_INVALID_ARGUMENT;
    }
    else
    {
        sdp_Error st = SDP_SUCCESS;
        if (tiles)
        {
            if (!occ) return SDP_ERR_RUNTIME;
            static_assert(32 * occ_classes(G) <= 320, "one bit per thread");
            k_row_occupancy<false><<<G / 64, 320, 0, stream>>>(tiles,
                    ncoarse, G, occ);
            SDP_HIP_CHECK_LAUNCH(&st);
            if (st) return st;
        }
        // One H row per workgroup iteration; Z formed in column pass A
        // (single-row form; the row-quad form measured 256 -> 242 us
        // for the row + column pass at config 2 and was removed).
        const size_t lds = row_lds_bytes(G);
        SDP_HIP_CHECK((allow_lds<k_rows_herm1<G>>(lds)), &st);
        if (st) return st;
        const int blocks = std::min(G / 2 + 1, num_cus() *
                (int)std::max<size_t>(1, (160 * 1024) / lds));
        k_rows_herm1<G><<<blocks, RowPlan<G>::P, lds, stream>>>(
                grid, g.k0, g.M, W, tiles ? occ : nullptr);
        SDP_HIP_CHECK_LAUNCH(&st);
        return st;
    }
}

template<int N1, int N2>
int grid_cols_a_herm(const Geometry& g, const float2* W, float2* grid,
        hipStream_t stream)
{
    constexpr int G = N1 * N2;
    if constexpr (G < 2048 || G > 8192)
    {
        return SDP_ERR_INVALID_ARGUMENT;
    }
    else
    {
        using HS = HalfSplit<G / 2>;
        sdp_Error st = SDP_SUCCESS;
        {
            constexpr int kTh = kPairsThreads;
            constexpr size_t kLds = kColLdsBytes * (kTh / 256);
            SDP_HIP_CHECK((allow_lds<k_cols_a_herm_pairs<HS::N1, HS::N2>>(
                    kLds)), &st);
            if (st) return st;
            const dim3 cg = col_grid<k_cols_a_herm_pairs<HS::N1, HS::N2>>(
                    HS::N1 / 2 + 1, g.M, kTh / ColPlan<HS::N2>::P, kTh, kLds,
                    kPairRounds);
            k_cols_a_herm_pairs<HS::N1, HS::N2><<<cg, kTh, kLds,
                    stream>>>(grid, g.M, W);
            SDP_HIP_CHECK_LAUNCH(&st);
            return st;
        }
    }
}

template<int N1, int N2>
int grid_to_image_herm(const Geometry& g, const ImageParams<float>& ip,
        const float2* W, const float2* grid, float* dirty, hipStream_t stream)
{
    constexpr int G = N1 * N2;
    if constexpr (G < 2048 || G > 8192)
    {
        return SDP_ERR_INVALID_ARGUMENT;
    }
    else
    {
        using HS = HalfSplit<G / 2>;
        sdp_Error st = SDP_SUCCESS;
        k_cols_b_herm<HS::N1, HS::N2><<<col_grid<k_cols_b_herm<HS::N1,
                HS::N2>>(HS::N2, g.M, ColPlan<HS::N1>::B), 256, kColLdsBytes,
                stream>>>(grid, dirty, ip, g.k0, g.M, W);
        SDP_HIP_CHECK_LAUNCH(&st);
        return st;
    }
}

template<int N1, int N2>
int image_cols_herm(const Geometry& g, const ImageParams<float>& ip,
        const float2* W, float* dirty, float2* grid, hipStream_t stream)
{
    constexpr int G = N1 * N2;
    if constexpr (G < 2048 || G > 8192)
    {
        return SDP_ERR_INVALID_ARGUMENT;
    }
    else
    {
        using HS = HalfSplit<G / 2>;
        sdp_Error st = SDP_SUCCESS;
        k_cols_a_image_herm<HS::N1, HS::N2><<<col_grid<k_cols_a_image_herm<
                HS::N1, HS::N2>>(HS::N1, g.M, ColPlan<HS::N2>::B), 256,
                kColLdsBytes, stream>>>(dirty, grid, ip, g.k0, g.M, W);
        SDP_HIP_CHECK_LAUNCH(&st);
        return st;
    }
}

template<int N1, int N2>
int image_to_grid_herm(const Geometry& g, const float2* W, float2* grid,
        const uint32_t* tiles, int ncoarse, uint32_t* need,
        hipStream_t stream)
{
    constexpr int G = N1 * N2;
    if constexpr (G < 2048 || G > 8192)
    {
        return SDP_ERR_INVALID_ARGUMENT;
    }
    else
    {
        using HS = HalfSplit<G / 2>;
        sdp_Error st = SDP_SUCCESS;
        if (tiles)
        {
            if (!need) return SDP_ERR_RUNTIME;
            k_row_occupancy<true><<<G / 64, 320, 0, stream>>>(tiles,
                    ncoarse, G, need);
            SDP_HIP_CHECK_LAUNCH(&st);
            if (st) return st;
        }
        {
            // X formed in column pass B; one row per workgroup iteration.
            const dim3 cg = col_grid<k_cols_b_image_herm_pairs<HS::N1,
                    HS::N2>>(HS::N2 / 2 + 1, g.M, ColPlan<HS::N1>::B, 256,
                    kColLdsBytes, kPairRounds);
            k_cols_b_image_herm_pairs<HS::N1, HS::N2><<<cg, 256,
                    kColLdsBytes, stream>>>(grid, g.M, W);
            SDP_HIP_CHECK_LAUNCH(&st);
            if (st) return st;
            const size_t lds = row_lds_bytes(G);
            SDP_HIP_CHECK((allow_lds<k_rows_image_herm1<G>>(lds)), &st);
            if (st) return st;
            const int blocks = std::min(G / 2 + 1, num_cus() *
                    (int)std::max<size_t>(1, (160 * 1024) / lds));
            k_rows_image_herm1<G><<<blocks, RowPlan<G>::P, lds, stream>>>(
                    grid, g.k0, g.M, W, tiles ? need : nullptr);
            SDP_HIP_CHECK_LAUNCH(&st);
            return st;
        }
    }
}

template<int N1, int N2>
int image_cols(const Geometry& g, const ImageParams<float>& ip, int plane,
        const float2* W, float* dirty, bool correct, float2* grid,
        hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    const dim3 blocks = ip.do_w ?
            col_grid<k_cols_a_image<N1, N2, true>>(N1, g.M, ColPlan<N2>::B) :
            col_grid<k_cols_a_image<N1, N2, false>>(N1, g.M, ColPlan<N2>::B);
    if (ip.do_w)
        k_cols_a_image<N1, N2, true><<<blocks, 256, kColLdsBytes, stream>>>(
                dirty, correct ? 1 : 0, grid, ip, plane, g.k0, g.M, W);
    else
        k_cols_a_image<N1, N2, false><<<blocks, 256, kColLdsBytes, stream>>>(
                dirty, correct ? 1 : 0, grid, ip, plane, g.k0, g.M, W);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<int N1, int N2>
int image_to_grid(const Geometry& g, const float2* W, float2* grid,
        const uint32_t* tiles, int ncoarse, hipStream_t stream)
{
    constexpr int G = N1 * N2;
    sdp_Error st = SDP_SUCCESS;
    k_cols_b_image<N1, N2><<<col_grid<k_cols_b_image<N1, N2>>(N2, g.M,
            ColPlan<N1>::B), 256,
            kColLdsBytes, stream>>>(grid, g.M, W);
    SDP_HIP_CHECK_LAUNCH(&st);
    if (st) return st;
    const size_t lds = row_lds_bytes(G);
    SDP_HIP_CHECK((allow_lds<k_rows_image<G>>(lds)), &st);
    if (st) return st;
    k_rows_image<G><<<row_blocks(G), RowPlan<G>::P, lds, stream>>>(
            grid, g.k0, g.M, W, tiles, ncoarse);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

// Whole-grid 2-D FFT in place, unnormalised (rocFFT / cuFFT convention:
// forward e^-, inverse e^+): rows, then the four-step columns; the output
// rows are stored permuted (k_cols_b_block).
template<int N1, int N2>
int fft2d_block(float2* grid, bool forward, const float2* W,
        hipStream_t stream)
{
    constexpr int G = N1 * N2;
    sdp_Error st = SDP_SUCCESS;
    const size_t lds = row_lds_bytes(G);
    if (forward)
    {
        SDP_HIP_CHECK((allow_lds<k_rows_image<G>>(lds)), &st);
        if (st) return st;
        k_rows_image<G><<<row_blocks(G), RowPlan<G>::P, lds, stream>>>(
                grid, 0, G, W, nullptr, 0);
        SDP_HIP_CHECK_LAUNCH(&st);
        if (st) return st;
        k_cols_a_grid<N1, N2, -1><<<col_grid<k_cols_a_grid<N1, N2, -1>>(N1,
                G, ColPlan<N2>::B), 256, kColLdsBytes, stream>>>(grid, G, W);
        SDP_HIP_CHECK_LAUNCH(&st);
        if (st) return st;
        k_cols_b_block<N1, N2, -1><<<col_grid<k_cols_b_block<N1, N2, -1>>(
                N2, G, ColPlan<N1>::B), 256, kColLdsBytes, stream>>>(grid, G,
                W);
    }
    else
    {
        SDP_HIP_CHECK((allow_lds<k_rows_grid<G>>(lds)), &st);
        if (st) return st;
        k_rows_grid<G><<<row_blocks(G), RowPlan<G>::P, lds, stream>>>(
                grid, 0, G, W, nullptr, 0);
        SDP_HIP_CHECK_LAUNCH(&st);
        if (st) return st;
        k_cols_a_grid<N1, N2, 1><<<col_grid<k_cols_a_grid<N1, N2, 1>>(N1,
                G, ColPlan<N2>::B), 256, kColLdsBytes, stream>>>(grid, G, W);
        SDP_HIP_CHECK_LAUNCH(&st);
        if (st) return st;
        k_cols_b_block<N1, N2, 1><<<col_grid<k_cols_b_block<N1, N2, 1>>(
                N2, G, ColPlan<N1>::B), 256, kColLdsBytes, stream>>>(grid, G,
                W);
    }
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

// Inverse FFT of a w-stack plane with the image update fused into the
// last column pass.
template<int N1, int N2>
int wstack_grid_image(float2* grid, const sdp_wt::AnyView& image, float norm,
        const sdp_wt::CorrParams& cp, const float2* W, hipStream_t stream)
{
    constexpr int G = N1 * N2;
    sdp_Error st = SDP_SUCCESS;
    const size_t lds = row_lds_bytes(G);
    SDP_HIP_CHECK((allow_lds<k_rows_grid<G>>(lds)), &st);
    if (st) return st;
    k_rows_grid<G><<<row_blocks(G), RowPlan<G>::P, lds, stream>>>(
            grid, 0, G, W, nullptr, 0);
    SDP_HIP_CHECK_LAUNCH(&st);
    if (st) return st;
    k_cols_a_grid<N1, N2, 1><<<col_grid<k_cols_a_grid<N1, N2, 1>>(N1, G,
            ColPlan<N2>::B), 256, kColLdsBytes, stream>>>(grid, G, W);
    SDP_HIP_CHECK_LAUNCH(&st);
    if (st) return st;
#define SDP_WS_COLB(IK) \
    k_cols_b_wstack_image<N1, N2, IK><<<col_grid<k_cols_b_wstack_image<N1, \
            N2, IK>>(N2, G, ColPlan<N1>::B), 256, kColLdsBytes, stream>>>( \
            grid, image.ptr, norm, cp, W)
    switch (image.kind)
    {
    case 0: SDP_WS_COLB(0); break;
    case 1: SDP_WS_COLB(1); break;
    case 2: SDP_WS_COLB(2); break;
    case 3: SDP_WS_COLB(3); break;
    default: return SDP_ERR_INVALID_ARGUMENT;
    }
#undef SDP_WS_COLB
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

// Sub-grid transforms of the w-towers imager --------------------------------
//
// Batched S x S complex-float 2-D FFTs (S = 128 or 256), unnormalised, in
// place in a sub-grid stack [slots][S][S] (sdp_grid_wstack_wtower.hip; the
// reference runs one 2-D FFT per sub-grid, sdp_grid_wstack_wtower.cpp:
// 686-711 via sdp_gridder_wtower_uvw.cpp). Two HBM passes instead of
// rocFFT's batched plan (whose column kernel ran at ~3.5 TB/s):
//  columns: length-S transforms of B = 256 / (S / 16) adjacent columns per
//           workgroup (ColFft, LDS e * B + column); in degridding the input
//           comes straight from the FFT'd w-stack plane (the sub-grid cut-out
//           of utils.cpp:603-649 with its checkerboard), which removes the
//           separate cut-out pass and its sub-grid-sized write and re-read;
//  rows   : B rows per workgroup, S / 16 consecutive lanes per row (each
//           load / store instruction moves whole 128-byte row segments),
//           LDS rows padded as RowIdx.
template<int S>
struct SubRowIdx
{
    static constexpr int kPitch = S + S / 16 + 8;
    int c;
    __device__ __forceinline__ int base(int b) const
    {
        return c * kPitch + b + (b >> 4);
    }
    static constexpr int off(int e) { return e + (e >> 4); }
};

template<int S, int SIGN, bool CUT>
__global__ void __launch_bounds__(256) k_sub_cols(float2* __restrict__ sub,
        const float2* __restrict__ W, SubgridCut cut)
{
    using F = ColFft<S, SIGN>;
    constexpr int B = ColPlan<S>::B, NCB = S / B;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    F f;
    f.init(p, W, S);
    const int64_t slot = blockIdx.x / NCB;
    const int col = (int)(blockIdx.x % NCB) * B + c;
    float2* s = sub + slot * S * S;
    float2 v[F::EPT];
    if constexpr (CUT)
    {
        // The slot's sub-grid origin in the plane grid (k_cut_out); G even,
        // so the checkerboard sign (gu + gv + a + b) & 1 of every element
        // is (ou + ov) & 1. Rows of the plane FFT are stored permuted.
        const int G = cut.G;
        const int t = cut.task[slot];
        const int q = t / cut.nv;
        const int iu = cut.min_iu + q, iv = cut.min_iv + (t - q * cut.nv);
        int ou = (G / 2 - S / 2 + iu * cut.eff) % G;
        int ov = (G / 2 - S / 2 + iv * cut.eff) % G;
        if (ou < 0) ou += G;
        if (ov < 0) ov += G;
        int gv = ov + col;
        if (gv >= G) gv -= G;
        const float sg = ((ou + ov) & 1) ? -1.0f : 1.0f;
        const int sh = cut.perm_shift;
        const unsigned n2m = sh >= 0 ? (1u << sh) - 1u : 0u;
        const unsigned n1 = sh >= 0 ? (unsigned)G >> sh : 0u;
        F::load_input(v, [&](int e) {
            int gu = ou + p + e;
            if (gu >= G) gu -= G;
            const unsigned r = sh >= 0 ? ((unsigned)gu & n2m) * n1 +
                    ((unsigned)gu >> sh) : (unsigned)gu;
            const float2 x = cut.grid[(size_t)r * G + gv];
            return make_float2(sg * x.x, sg * x.y);
        });
    }
    else
    {
        F::load_input(v, [&](int e) { return s[(p + e) * S + col]; });
    }
    f.transform(v, p, lds, ColIdx<B>{c});
    F::store_output(v, [&](int e, int, float2 x) { s[(p + e) * S + col] = x; });
}

template<int S, int SIGN>
__global__ void __launch_bounds__(256) k_sub_rows(float2* __restrict__ sub,
        const float2* __restrict__ W)
{
    using F = ColFft<S, SIGN>;
    constexpr int P = ColPlan<S>::P, B = ColPlan<S>::B;
    extern __shared__ float2 lds[];
    const int p = threadIdx.x % P, c = threadIdx.x / P;
    F f;
    f.init(p, W, S);
    float2* r = sub + ((int64_t)blockIdx.x * B + c) * S;
    float2 v[F::EPT];
    F::load_input(v, [&](int e) { return r[p + e]; });
    f.transform(v, p, lds, SubRowIdx<S>{c});
    F::store_output(v, [&](int e, int, float2 x) { r[p + e] = x; });
}

template<int S>
int subgrid_fft_s(float2* sub, int64_t slots, bool forward, const float2* W,
        const SubgridCut* cut, hipStream_t stream)
{
    constexpr int B = ColPlan<S>::B;
    sdp_Error st = SDP_SUCCESS;
    if (slots <= 0) return st;
    const size_t rl = (size_t)B * SubRowIdx<S>::kPitch * sizeof(float2);
    // One workgroup per column block / row block (a persistent form with
    // 4 or 8 workgroups per CU measured the same at config 4).
    const unsigned ncol = (unsigned)(slots * (S / B));
    const unsigned nrow = ncol;
    if (forward)
    {
        k_sub_cols<S, -1, false><<<ncol, 256, kColLdsBytes, stream>>>(sub, W,
                SubgridCut{});
        SDP_HIP_CHECK_LAUNCH(&st);
        if (st) return st;
        k_sub_rows<S, -1><<<nrow, 256, rl, stream>>>(sub, W);
    }
    else
    {
        if (cut)
            k_sub_cols<S, 1, true><<<ncol, 256, kColLdsBytes, stream>>>(sub,
                    W, *cut);
        else
            k_sub_cols<S, 1, false><<<ncol, 256, kColLdsBytes, stream>>>(sub,
                    W, SubgridCut{});
        SDP_HIP_CHECK_LAUNCH(&st);
        if (st) return st;
        k_sub_rows<S, 1><<<nrow, 256, rl, stream>>>(sub, W);
    }
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

// Forward FFT of a w-stack plane from its image (degridding prologue):
// columns (image prologue) first, then rows.
template<int N1, int N2>
int wstack_image_to_grid(float2* grid, const sdp_wt::AnyView& image,
        const sdp_wt::CorrParams& cp, const float2* W, hipStream_t stream)
{
    constexpr int G = N1 * N2;
    sdp_Error st = SDP_SUCCESS;
#define SDP_WS_COLA(IK) \
    k_cols_a_wstack_image<N1, N2, IK><<<col_grid<k_cols_a_wstack_image<N1, \
            N2, IK>>(N1, G, ColPlan<N2>::B), 256, kColLdsBytes, stream>>>( \
            grid, image.ptr, cp, W)
    switch (image.kind)
    {
    case 0: SDP_WS_COLA(0); break;
    case 1: SDP_WS_COLA(1); break;
    case 2: SDP_WS_COLA(2); break;
    case 3: SDP_WS_COLA(3); break;
    default: return SDP_ERR_INVALID_ARGUMENT;
    }
#undef SDP_WS_COLA
    SDP_HIP_CHECK_LAUNCH(&st);
    if (st) return st;
    k_cols_b_block<N1, N2, -1><<<col_grid<k_cols_b_block<N1, N2, -1>>(N2, G,
            ColPlan<N1>::B), 256, kColLdsBytes, stream>>>(grid, G, W);
    SDP_HIP_CHECK_LAUNCH(&st);
    if (st) return st;
    const size_t lds = row_lds_bytes(G);
    SDP_HIP_CHECK((allow_lds<k_rows_image<G>>(lds)), &st);
    if (st) return st;
    k_rows_image<G><<<row_blocks(G), RowPlan<G>::P, lds, stream>>>(grid, 0,
            G, W, nullptr, 0);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

// Dispatch on G = N1 * N2 (N2 = N1 or 2 * N1).
#define SDP_ES_FFT_DISPATCH(G, CALL) \
    switch (G) \
    { \
    case 1024:  { constexpr int N1 = 32,  N2 = 32;  return CALL; } \
    case 2048:  { constexpr int N1 = 32,  N2 = 64;  return CALL; } \
    case 4096:  { constexpr int N1 = 64,  N2 = 64;  return CALL; } \
    case 8192:  { constexpr int N1 = 64,  N2 = 128; return CALL; } \
    case 16384: { constexpr int N1 = 128, N2 = 128; return CALL; } \
    default: return SDP_ERR_INVALID_ARGUMENT; \
    }

} // namespace

bool fused_fft_supported(int grid_size)
{
    switch (grid_size)
    {
    case 1024: case 2048: case 4096: case 8192: case 16384:
        return true;
    default:
        return false;
    }
}

int fft_twiddles_create(int grid_size, FftTwiddles* tw)
{
    sdp_Error st = SDP_SUCCESS;
    std::vector<float2> h((size_t)grid_size);
    for (int m = 0; m < grid_size; ++m)
    {
        const double a = kTwoPi * (double)m / (double)grid_size;
        h[m] = make_float2((float)std::cos(a), (float)(-std::sin(a)));
    }
    SDP_HIP_CHECK(hipMalloc(&tw->table, h.size() * sizeof(float2)), &st);
    if (st) return st;
    SDP_HIP_CHECK(hipMemcpy(tw->table, h.data(), h.size() * sizeof(float2),
            hipMemcpyHostToDevice), &st);
    if (!st && grid_size >= 2048)
        SDP_HIP_CHECK(hipMalloc(&tw->masks, (size_t)(grid_size / 64) *
                occ_classes(grid_size) * sizeof(uint32_t)), &st);
    tw->G = grid_size;
    return st;
}

void fft_twiddles_destroy(FftTwiddles* tw)
{
    if (tw->table) (void)hipFree(tw->table);
    if (tw->masks) (void)hipFree(tw->masks);
    tw->table = nullptr;
    tw->masks = nullptr;
    tw->G = 0;
}

int fft_grid_rows(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
    if (herm_enabled(ip))
        SDP_ES_FFT_DISPATCH(g.G, (grid_rows_herm<N1, N2>(g, W,
                (float2*)grid, tiles, ncoarse, (uint32_t*)tw.masks, stream)))
    SDP_ES_FFT_DISPATCH(g.G, (grid_rows<N1, N2>(g, W, (float2*)grid,
            tiles, ncoarse, stream)))
}

int fft_grid_cols_a(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
    if (herm_enabled(ip))
        SDP_ES_FFT_DISPATCH(g.G, (grid_cols_a_herm<N1, N2>(g, W,
                (float2*)grid, stream)))
    SDP_ES_FFT_DISPATCH(g.G, (grid_cols_a<N1, N2>(g, W, (float2*)grid,
            stream)))
}

int fft_grid_rows_cols(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, hipStream_t stream)
{
    const int e = fft_grid_rows(ip, tw, grid, tiles, ncoarse, stream);
    return e ? e : fft_grid_cols_a(ip, tw, grid, stream);
}

void fft_grid_row_spectra(const ImageParams<float>& ip, int64_t* rows,
        int64_t* col0, int64_t* ncols)
{
    const Geometry g = geometry(ip);
    // The row passes store a row's M centre outputs at columns [0, M)
    // (k_rows_grid, k_rows_herm1: buffer base grid - k0).
    *rows = herm_enabled(ip) ? g.G / 2 + 1 : g.G;
    *col0 = 0;
    *ncols = g.M;
}

int fft_grid_to_image(const ImageParams<float>& ip, int plane,
        const FftTwiddles& tw, float* grid, float* dirty, hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
    if (herm_enabled(ip))
        SDP_ES_FFT_DISPATCH(g.G, (grid_to_image_herm<N1, N2>(g, ip, W,
                (const float2*)grid, dirty, stream)))
    SDP_ES_FFT_DISPATCH(g.G, (grid_to_image<N1, N2>(g, ip, plane, W,
            (const float2*)grid, dirty, stream)))
}

bool fft_degrid_real_form(const ImageParams<float>& ip,
        bool correct_in_place)
{
    return herm_degrid_enabled(ip) && correct_in_place;
}

int fft_image_cols(const ImageParams<float>& ip, int plane,
        const FftTwiddles& tw, float* dirty, bool correct_in_place,
        bool real_form, float* grid, hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
    // The real-input form corrects the image in place in its prologue and
    // exists for the 2-D grids herm_degrid_enabled accepts only.
    if (real_form && !fft_degrid_real_form(ip, correct_in_place))
        return SDP_ERR_INVALID_ARGUMENT;
    if (real_form)
        SDP_ES_FFT_DISPATCH(g.G, (image_cols_herm<N1, N2>(g, ip, W, dirty,
                (float2*)grid, stream)))
    SDP_ES_FFT_DISPATCH(g.G, (image_cols<N1, N2>(g, ip, plane, W, dirty,
            correct_in_place, (float2*)grid, stream)))
}

int fft_image_to_grid(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, bool real_form,
        hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
    if (real_form && !herm_degrid_enabled(ip)) return SDP_ERR_INVALID_ARGUMENT;
    if (real_form)
        SDP_ES_FFT_DISPATCH(g.G, (image_to_grid_herm<N1, N2>(g, W,
                (float2*)grid, tiles, ncoarse, (uint32_t*)tw.masks, stream)))
    SDP_ES_FFT_DISPATCH(g.G, (image_to_grid<N1, N2>(g, W, (float2*)grid,
            tiles, ncoarse, stream)))
}

int fft2d_inplace_permuted(float* grid, int grid_size, bool forward,
        const FftTwiddles& tw, hipStream_t stream)
{
    if (tw.G != grid_size) return SDP_ERR_INVALID_ARGUMENT;
    const float2* W = (const float2*)tw.table;
    SDP_ES_FFT_DISPATCH(grid_size, (fft2d_block<N1, N2>((float2*)grid,
            forward, W, stream)))
}

int fft2d_wstack_grid_image(float* grid, int grid_size, const FftTwiddles& tw,
        const sdp_wt::AnyView& image, float norm,
        const sdp_wt::CorrParams& cp, hipStream_t stream)
{
    if (tw.G != grid_size) return SDP_ERR_INVALID_ARGUMENT;
    const float2* W = (const float2*)tw.table;
    SDP_ES_FFT_DISPATCH(grid_size, (wstack_grid_image<N1, N2>((float2*)grid,
            image, norm, cp, W, stream)))
}

int fft2d_wstack_image_to_grid(float* grid, int grid_size,
        const FftTwiddles& tw, const sdp_wt::AnyView& image,
        const sdp_wt::CorrParams& cp, hipStream_t stream)
{
    if (tw.G != grid_size) return SDP_ERR_INVALID_ARGUMENT;
    const float2* W = (const float2*)tw.table;
    SDP_ES_FFT_DISPATCH(grid_size, (wstack_image_to_grid<N1, N2>(
            (float2*)grid, image, cp, W, stream)))
}

bool subgrid_fft_supported(int subgrid_size)
{
    return subgrid_size == 128 || subgrid_size == 256;
}

int subgrid_fft2d(float* sub, int subgrid_size, int64_t slots, bool forward,
        const FftTwiddles& tw, const SubgridCut* cut, hipStream_t stream)
{
    if (tw.G != subgrid_size || slots * subgrid_size > INT32_MAX ||
            (cut && (cut->G % 2 != 0 || cut->G < subgrid_size)))
        return SDP_ERR_INVALID_ARGUMENT;
    const float2* W = (const float2*)tw.table;
    switch (subgrid_size)
    {
    case 128: return subgrid_fft_s<128>((float2*)sub, slots, forward, W, cut,
            stream);
    case 256: return subgrid_fft_s<256>((float2*)sub, slots, forward, W, cut,
            stream);
    default: return SDP_ERR_INVALID_ARGUMENT;
    }
}

int fft_perm_n2(int grid_size)
{
    switch (grid_size)
    {
    case 1024: return 32;
    case 2048: return 64;
    case 4096: return 64;
    case 8192: return 128;
    case 16384: return 128;
    default: return 0;
    }
}

} // namespace sdp_es
