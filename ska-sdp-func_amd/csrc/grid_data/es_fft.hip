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
#include <cmath>
#include <utility>
#include <vector>

#include "es_fft.h"
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
#ifndef SDP_COLA_WAVES
#define SDP_COLA_WAVES 4
#endif
#ifndef SDP_COLB_WAVES
#define SDP_COLB_WAVES 3
#endif

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
                float re, im;
                phasor(ip, plane, abs(xo), abs(yo), -1.0f, re, im);
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

// Split of the half-length column transform, G2 = N1 * N2.
template<int G2> struct HalfSplit;
template<> struct HalfSplit<1024> { static constexpr int N1 = 32, N2 = 32; };
template<> struct HalfSplit<2048> { static constexpr int N1 = 32, N2 = 64; };
template<> struct HalfSplit<4096> { static constexpr int N1 = 64, N2 = 64; };
template<> struct HalfSplit<8192> { static constexpr int N1 = 64, N2 = 128; };

__host__ __device__ constexpr int mask_words(int G)
{
    return G / 64 > 64 ? G / 4096 : 1;
}

// Occupied-tile bitmap: word w of tile row tu has bit b set if tile
// 64 w + b of that row holds bucketed entries (one 64-thread block per
// tile row).
__global__ void __launch_bounds__(64) k_tile_masks(
        const uint32_t* __restrict__ tiles, int ncoarse, int ntiles,
        int words, uint64_t* __restrict__ masks)
{
    const unsigned tu = blockIdx.x;
    for (int w = 0; w < words; ++w)
    {
        const unsigned tv = (unsigned)(64 * w) + threadIdx.x;
        bool occ = false;
        if (tv < (unsigned)ntiles)
        {
            const unsigned bin = (((tu >> 2) * (unsigned)ncoarse + (tv >> 2))
                    << 4) | ((tu & 3u) << 2) | (tv & 3u);
            occ = tiles[bin] != 0u;
        }
        const uint64_t m = __ballot(occ);
        if (threadIdx.x == 0) masks[tu * words + w] = m;
    }
}

template<int G>
__global__ void __launch_bounds__(RowPlan<G>::P)
k_rows_herm(float2* __restrict__ grid, int k0, int M,
        const float2* __restrict__ W, const uint64_t* __restrict__ masks)
{
    using F = RowFft<G, 1>;
    constexpr int EPT = F::EPT, NW = mask_words(G), NQ = G / 4 + 1;
    extern __shared__ float2 lds[];
    const int p = threadIdx.x;
    const Buf gb(grid - k0, grid_bytes(G, k0));
    F f;
    f.init(p, W, G);
    const int per = (NQ + gridDim.x - 1) / gridDim.x;
    const int q_begin = blockIdx.x * per, q_end = min(NQ, q_begin + per);
    // H row u from grid rows u and -u (element v and -v); tiles with no
    // bucketed entry were not written by the scatter and read as zero.
    auto load_h = [&](float2 (&v)[EPT], int u, int pq) {
        const int ur = (G - u) & (G - 1);
        uint64_t wa[NW], wb[NW];
#pragma unroll
        for (int w = 0; w < NW; ++w)
        {
            wa[w] = masks ? masks[(u >> 6) * NW + w] : ~0ull;
            wb[w] = masks ? masks[(ur >> 6) * NW + w] : ~0ull;
        }
        const uint32_t ra = ((uint32_t)u * G + k0) * 8u;
        const uint32_t rb = ((uint32_t)ur * G + k0) * 8u;
        F::load_input(v, [&](int c) {
            const int ca = pq + c, cb = (G - ca) & (G - 1);
            const int ta = ca >> 6, tb = cb >> 6;
            const bool oa = (wa[NW > 1 ? ta >> 6 : 0] >> (ta & 63)) & 1ull;
            const bool ob = (wb[NW > 1 ? tb >> 6 : 0] >> (tb & 63)) & 1ull;
            const float2 a = gb.load_if(oa, ra + (uint32_t)ca * 8u);
            const float2 b = gb.load_if(ob, rb + (uint32_t)cb * 8u);
            return make_float2(0.5f * (a.x + b.x), 0.5f * (a.y - b.y));
        });
    };
    for (int k = q_begin; k < q_end; ++k)
    {
        const int pq = opaque(p);
        const int ub = G / 2 - k;              // == k for the quad k = G/4
        float2 va[EPT], vb[EPT];
        load_h(va, k, pq);
        f.transform(va, pq, lds, RowIdx{});
        if (ub != k)
        {
            load_h(vb, ub, pq);
            f.transform(vb, pq, lds, RowIdx{});
        }
        else
        {
#pragma unroll
            for (int i = 0; i < EPT; ++i) vb[i] = va[i];
        }
        // e^{2 pi i k / G} = conj(W[k]); e^{2 pi i (G/2 - k) / G} = -W[k].
        const float2 wt = W[k];
        const float2 wk = make_float2(wt.x, -wt.y);
        const float2 wb = make_float2(-wt.x, -wt.y);
        float2 za[EPT];
#pragma unroll
        for (int i = 0; i < EPT; ++i)
        {
            const float2 a = va[i], b = vb[i];
            const float2 xe = make_float2(a.x + b.x, a.y - b.y);
            const float2 xo = cmul(make_float2(a.x - b.x, a.y + b.y), wk);
            za[i] = make_float2(xe.x - xo.y, xe.y + xo.x);
            // Z[G/2 - k] from the same pair, roles swapped.
            const float2 ye = make_float2(b.x + a.x, b.y - a.y);
            const float2 yo = cmul(make_float2(b.x - a.x, b.y + a.y), wb);
            vb[i] = make_float2(ye.x - yo.y, ye.y + yo.x);
        }
        const uint32_t vo = (uint32_t)pq * 8u;
        const uint32_t va_row = (uint32_t)k * G * 8u + vo;
        F::store_output(za, [&](int c, int, float2 x) {
            gb.store_if((unsigned)(pq + c - k0) < (unsigned)M, x, va_row + c * 8u);
        });
        if (k > 0 && ub != k)
        {
            const uint32_t vb_row = (uint32_t)ub * G * 8u + vo;
            F::store_output(vb, [&](int c, int, float2 x) {
                gb.store_if((unsigned)(pq + c - k0) < (unsigned)M, x,
                        vb_row + c * 8u);
            });
        }
    }
}

// Column pass A of the half-length transform: for u1 = blockIdx.x,
// length-N2 FFTs over the Z rows u1 + N1 * n2 (row pitch G = 2 N1 N2),
// times e^{2 pi i u1 k2 / (G/2)}, back into rows u1 + N1 * k2.
template<int N1, int N2>
__global__ void __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(SDP_COLA_WAVES)))
k_cols_a_herm(float2* __restrict__ grid, int M, const float2* __restrict__ W)
{
    constexpr int G = 2 * N1 * N2, B = ColPlan<N2>::B;
    using F = ColFft<N2, 1>;
    extern __shared__ float2 lds[];
    const int c = threadIdx.x % B, p = threadIdx.x / B;
    const int u1 = blockIdx.x;
    const Buf gb(grid, grid_bytes(G, 0));
    F f;
    f.init(p, W, G);
    float2 fs[F::EPT];
#pragma unroll
    for (int i = 0; i < F::EPT; ++i)
        fs[i] = F::twiddle(W, 2 * u1 * F::out_index(p, i));
    const int ncb = (M + B - 1) / B;
    const uint32_t so = (uint32_t)u1 * G * 8u;
    constexpr uint32_t kStep = (uint32_t)N1 * G * 8u;
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
            if constexpr (DO_W)
                phasor(ip, plane, abs(xo), abs(yo), 1.0f, pr, pi);
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

// Column-pass workgroups: rounds x the kernel's resident workgroups per CU
// (env SDP_ES_COL_ROUNDS for experiments; default 2). A launch that is not
// a whole number of resident rounds leaves its last round partly empty:
// 4 per CU for the kernels that hold 3 (VGPRs) cost config 2 0.03 ms of
// grid FFT + image and 0.05 ms of degrid FFT; the degrid column pass B
// holds 5 (LDS) and ran 1.2 rounds at 6 per CU.
int col_rounds()
{
    static int v = 0;
    if (!v)
    {
        const char* e = getenv("SDP_ES_COL_ROUNDS");
        v = e ? std::max(1, atoi(e)) : 2;
    }
    return v;
}

template<auto Kernel>
dim3 col_grid(int fixed, int M, int B)
{
    static int occ = 0;
    if (!occ)
    {
        int n = 0;
        if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&n, Kernel, 256,
                kColLdsBytes) != hipSuccess || n <= 0)
            n = 3;
        occ = n;
    }
    const int ncb = (M + B - 1) / B;
    const int want = num_cus() * occ * col_rounds();
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
int grid_rows_cols(const Geometry& g, const float2* W, float2* grid,
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
    if (st) return st;
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
    const dim3 blocks = ip.do_w ?
            col_grid<k_cols_b_grid<N1, N2, true>>(N2, g.M, ColPlan<N1>::B) :
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
// 2048 to 8192 (at 16384 the row pass's two 32-element rows per thread do
// not fit the registers; env SDP_ES_HERM=0: the complex form, for A/B).
bool herm_enabled(const ImageParams<float>& ip)
{
    static int on = -1;
    if (on < 0)
    {
        const char* e = getenv("SDP_ES_HERM");
        on = (e && e[0] == '0') ? 0 : 1;
    }
    return on && !ip.do_w && ip.G >= 2048 && ip.G <= 8192;
}

template<int N1, int N2>
int grid_rows_cols_herm(const Geometry& g, const float2* W, float2* grid,
        const uint32_t* tiles, int ncoarse, uint64_t* masks,
        hipStream_t stream)
{
    constexpr int G = N1 * N2;
    if constexpr (G < 2048)
    {
        return SDP_ERR_INVALID_ARGUMENT;
    }
    else
    {
        using HS = HalfSplit<G / 2>;
        sdp_Error st = SDP_SUCCESS;
        if (tiles)
        {
            if (!masks) return SDP_ERR_RUNTIME;
            k_tile_masks<<<G / 64, 64, 0, stream>>>(tiles, ncoarse, G / 64,
                    mask_words(G), masks);
            SDP_HIP_CHECK_LAUNCH(&st);
            if (st) return st;
        }
        const size_t lds = row_lds_bytes(G);
        SDP_HIP_CHECK((allow_lds<k_rows_herm<G>>(lds)), &st);
        if (st) return st;
        k_rows_herm<G><<<row_blocks(G), RowPlan<G>::P, lds, stream>>>(
                grid, g.k0, g.M, W, tiles ? masks : nullptr);
        SDP_HIP_CHECK_LAUNCH(&st);
        if (st) return st;
        k_cols_a_herm<HS::N1, HS::N2><<<col_grid<k_cols_a_herm<HS::N1,
                HS::N2>>(HS::N1, g.M, ColPlan<HS::N2>::B), 256, kColLdsBytes,
                stream>>>(grid, g.M, W);
        SDP_HIP_CHECK_LAUNCH(&st);
        return st;
    }
}

template<int N1, int N2>
int grid_to_image_herm(const Geometry& g, const ImageParams<float>& ip,
        const float2* W, const float2* grid, float* dirty, hipStream_t stream)
{
    constexpr int G = N1 * N2;
    if constexpr (G < 2048)
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
                mask_words(grid_size) * sizeof(uint64_t)), &st);
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

int fft_grid_rows_cols(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
    if (herm_enabled(ip))
        SDP_ES_FFT_DISPATCH(g.G, (grid_rows_cols_herm<N1, N2>(g, W,
                (float2*)grid, tiles, ncoarse, (uint64_t*)tw.masks, stream)))
    SDP_ES_FFT_DISPATCH(g.G, (grid_rows_cols<N1, N2>(g, W, (float2*)grid,
            tiles, ncoarse, stream)))
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

int fft_image_cols(const ImageParams<float>& ip, int plane,
        const FftTwiddles& tw, float* dirty, bool correct_in_place,
        float* grid, hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
    SDP_ES_FFT_DISPATCH(g.G, (image_cols<N1, N2>(g, ip, plane, W, dirty,
            correct_in_place, (float2*)grid, stream)))
}

int fft_image_to_grid(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, hipStream_t stream)
{
    const Geometry g = geometry(ip);
    const float2* W = (const float2*)tw.table;
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
