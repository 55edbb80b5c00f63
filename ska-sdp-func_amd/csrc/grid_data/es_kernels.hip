// HIP kernels of the MI355X-native ES-FFT (de)gridder. See es_kernels.h for
// the data path. Per-visibility arithmetic (positions, tap ranges, the
// exponential-of-semicircle taps, checkerboard sign, w<0 flip) follows the
// reference kernels sdp_gridder_uvw_es_fft_kernels.cu:97-422 operation for
// operation, in the same precision, so taps match the reference bit-for-bit
// up to the libm exp/sqrt ulp; only the summation ORDER differs (LDS tile
// accumulation instead of per-tap HBM atomics).
#include <cmath>
#include <cstdlib>
#include <cstring>

#include "utility/wave_ops.h"
#include "es_kernels.h"
#include "es_params.h"
#include "es_image_dev.h"
#include "../utility/sdp_hip.h"

namespace sdp_es {
namespace {

using img::inv_correction;
using img::phasor;

constexpr double kSpeedOfLight = 299792458.0;
constexpr int kThreads = 256;
constexpr int kWaves = kThreads / 64;
constexpr int kScatterStride = kTile + 8;   // 72 = 8 (mod 32): conflict-free

template<typename T> struct Vec2;
template<> struct Vec2<float> { using type = float2; };
template<> struct Vec2<double> { using type = double2; };

// Exponential of semicircle, kernels.cu:97-102.
template<typename T>
__device__ __forceinline__ T es_tap(T beta, T x)
{
#pragma clang fp contract(off)
    const T xx = x * x;
    return (xx > T(1)) ? T(0) : exp(beta * (sqrt(T(1) - xx) - T(1)));
}

// Exponential of semicircle on the hardware transcendental units, for the
// f32 matrix-core kernels: v_sqrt_f32 (1 ulp; the argument 1 - x^2 lies in
// [6e-8, 1], never denormal) and exp(y) = 2^(y log2 e) with the rounding
// error of y log2 e fed back to first order (|error| ~ 1-2 ulp over the
// kernel's range |y| <= beta ~ 16). Same formula and branch as es_tap;
// the taps differ from libm's correctly rounded ones by ~1e-7 relative.
__device__ __forceinline__ float es_tap_fast(float beta, float x)
{
#pragma clang fp contract(off)
    const float xx = x * x;
    const float y = beta * (__builtin_amdgcn_sqrtf(1.0f - xx) - 1.0f);
    const float t = y * 1.44269504088896341f;
    const float err = __builtin_fmaf(y, 1.44269504088896341f, -t) +
            y * 1.92596299112661746e-8f;
    const float e = __builtin_amdgcn_exp2f(t);
    const float r = __builtin_fmaf(e, err * 0.693147180559945309f, e);
    return (xx > 1.0f) ? 0.0f : r;
}

// Taps of one axis of a bucketed entry for the f32 tile kernels: slot d
// holds the tap at u0 + d (u0 the clamped first tap, zero past u1), with
// the checkerboard factor (-1)^d of the slot (the entry's (-1)^u0 is
// applied by the caller). kernels.cu:97-102 evaluates every tap as
// exp(beta (sqrt(1 - x^2) - 1)); here, for W = 8 and an unclamped first
// tap, the two edge taps (d = 0, 7: the sqrt branch point makes them
// non-polynomial) and the exact-integer ninth tap are evaluated that way,
// and the six interior taps (smooth in delta = u0 - (pos - 4) in [0, 1))
// as degree-8 polynomials of s = 2 delta - 1 in packed-f32 Horner form,
// two taps per v_pk_fma_f32 (~9e-8 absolute in f32, es_tap_poly_fit):
// 3 exp/sqrt pairs per axis instead of 9.
template<int NTAP, bool POLY>
__device__ __forceinline__ void axis_taps(const EsParams<float>& p, float pos,
        int u0, int u1, float (&t)[NTAP])
{
#pragma clang fp contract(off)
    using f2 = __attribute__((ext_vector_type(2))) float;
    const float hs = (float)p.support / 2.0f;
    const float inv_hs = 1.0f / hs;
    if (POLY && NTAP == 9 && p.tap_poly_ok && u1 >= u0 + 7 &&
            u0 == (int)ceilf(pos - hs))
    {
        const float dl = ((float)u0 - pos) + hs;    // exact, in [0, 1)
        const float sv = dl * 2.0f - 1.0f;           // exact
        const f2 s2 = {sv, sv};
#pragma unroll
        for (int q = 0; q < kTapPolyPairs; ++q)
        {
            f2 y = {p.tap_poly[q][kTapPolyDeg][0], p.tap_poly[q][kTapPolyDeg][1]};
#pragma unroll
            for (int k = kTapPolyDeg - 1; k >= 0; --k)
            {
                const f2 c = {p.tap_poly[q][k][0], p.tap_poly[q][k][1]};
                y = __builtin_elementwise_fma(y, s2, c);
            }
            t[1 + 2 * q] = y.x;
            t[2 + 2 * q] = y.y;
        }
        t[0] = es_tap_fast(p.beta, ((float)u0 - pos) * inv_hs);
        t[7] = -es_tap_fast(p.beta, ((float)(u0 + 7) - pos) * inv_hs);
        t[8] = 0.0f;
        if (u1 >= u0 + 8)   // exact-integer position: W + 1 taps
            t[NTAP - 1] = es_tap_fast(p.beta,
                    ((float)(u0 + 8) - pos) * inv_hs);
        return;
    }
#pragma unroll
    for (int d = 0; d < NTAP; ++d)
    {
        const float k = es_tap_fast(p.beta, ((float)(u0 + d) - pos) * inv_hs);
        t[d] = (u0 + d <= u1) ? ((d & 1) ? -k : k) : 0.0f;
    }
}

// Tap range of one visibility on the current w-plane (kernels.cu:150-196,
// 301-347). Returns false if the visibility does not touch the plane.
template<typename T>
struct Footprint
{
    T pu, pv, kw, flip;
    int u0, u1, v0, v1;
};

// iwl: freq / c of the visibility's channel. The reference's (flip * freq)
// / c (kernels.cu:163) with flip = +-1 equals +-(freq / c) exactly (IEEE
// division is sign-symmetric), so callers form the quotient once per
// channel where they can (chan_quotient).
template<typename T>
__device__ __forceinline__ bool footprint(const EsParams<T>& p, T u, T v,
        T w, T iwl, Footprint<T>& f)
{
#pragma clang fp contract(off)
    f.flip = (p.do_w && w < T(0)) ? T(-1) : T(1);
    const T inv_wavelength = f.flip < T(0) ? -iwl : iwl;
    const T half_support = T(p.support) / T(2);
    const int gmin = -p.G / 2, gmax = (p.G - 1) / 2;
    f.pu = u * inv_wavelength * p.uv_scale;
    f.pv = v * inv_wavelength * p.uv_scale;
    f.u0 = max((int)ceil(f.pu - half_support), gmin);
    f.u1 = min((int)floor(f.pu + half_support), gmax);
    f.v0 = max((int)ceil(f.pv - half_support), gmin);
    f.v1 = min((int)floor(f.pv + half_support), gmax);
    f.kw = T(1);
    if (p.do_w)
    {
        const T pos_w = (w * inv_wavelength - p.min_plane_w) * p.w_scale;
        if (p.plane < 0)
        {
            // Bucketing for every w-plane at once: the record keeps the
            // plane coordinate (> 0: min_plane_w lies W / 2 - 1 planes
            // below the smallest |w|); the tile kernel of plane p derives
            // the w-tap (plane_tap) and skips the planes it misses.
            f.kw = pos_w;
            return f.u0 <= f.u1 && f.v0 <= f.v1;
        }
        const int w0 = (int)ceil(pos_w - half_support);
        const int w1 = (int)floor(pos_w + half_support);
        if (p.plane < w0 || p.plane > w1) return false;
        const T inv_half_support = T(1) / half_support;
        f.kw = es_tap(p.beta, (T)(p.plane - pos_w) * inv_half_support);
    }
    return f.u0 <= f.u1 && f.v0 <= f.v1;
}

// w-tap of plane p.plane for a record bucketed for all planes (its plane
// coordinate pos_w, footprint() with p.plane < 0): the same arithmetic as
// footprint(); false (tap 0) if the visibility does not touch the plane.
template<typename T>
__device__ __forceinline__ bool plane_tap_at(const EsParams<T>& p, int plane,
        T pos_w, T& kw)
{
#pragma clang fp contract(off)
    const T half_support = T(p.support) / T(2);
    const int w0 = (int)ceil(pos_w - half_support);
    const int w1 = (int)floor(pos_w + half_support);
    kw = T(0);
    if (plane < w0 || plane > w1) return false;
    const T inv_half_support = T(1) / half_support;
    kw = es_tap(p.beta, (T)(plane - pos_w) * inv_half_support);
    return true;
}

template<typename T>
__device__ __forceinline__ bool plane_tap(const EsParams<T>& p, T pos_w,
        T& kw)
{
#pragma clang fp contract(off)
    const T half_support = T(p.support) / T(2);
    const int w0 = (int)ceil(pos_w - half_support);
    const int w1 = (int)floor(pos_w + half_support);
    kw = T(0);
    if (p.plane < w0 || p.plane > w1) return false;
    const T inv_half_support = T(1) / half_support;
    kw = es_tap(p.beta, (T)(p.plane - pos_w) * inv_half_support);
    return true;
}

// Clamped tap range from a record position (same formula as footprint()).
template<typename T>
__device__ __forceinline__ void tap_range(const EsParams<T>& p, T pu, T pv,
        int& u0, int& u1, int& v0, int& v1)
{
#pragma clang fp contract(off)
    const T half_support = T(p.support) / T(2);
    const int gmin = -p.G / 2, gmax = (p.G - 1) / 2;
    u0 = max((int)ceil(pu - half_support), gmin);
    u1 = min((int)floor(pu + half_support), gmax);
    v0 = max((int)ceil(pv - half_support), gmin);
    v1 = min((int)floor(pv + half_support), gmax);
}

template<typename T>
__device__ __forceinline__ T tap_weight(const EsParams<T>& p, int u, int v,
        T pu, T pv, T kw)
{
#pragma clang fp contract(off)
    const T inv_half_support = T(1) / (T(p.support) / T(2));
    const T ku = es_tap(p.beta, (T)(u - pu) * inv_half_support);
    const T kv = es_tap(p.beta, (T)(v - pv) * inv_half_support);
    T k = ku * kv * kw;
    return ((u + v) & 1) ? -k : k;
}

// Records ------------------------------------------------------------------

template<typename T, int MODE, bool DO_W>
struct Rec
{
    static constexpr int kWords = (MODE == MODE_GRID && DO_W) ? 8 : 4;
};

__device__ __forceinline__ float idx_bits(float, uint64_t i)
{
    return __uint_as_float((uint32_t)i);
}
__device__ __forceinline__ double idx_bits(double, uint64_t i)
{
    return __longlong_as_double((long long)i);
}
__device__ __forceinline__ uint64_t bits_idx(float x)
{
    return (uint64_t)__float_as_uint(x);
}
__device__ __forceinline__ uint64_t bits_idx(double x)
{
    return (uint64_t)__double_as_longlong(x);
}

// Bin b -> origin (row, col) of its 64 x 64 tile. Bins are numbered
// block-major: 16 per 4 x 4-tile block, row-major inside it, so the tile
// kernels' consecutive work items write / read adjacent tiles (measured
// 5 % faster tile kernels than row-major bins at config 2).
template<typename T>
__device__ __forceinline__ void tile_origin(const EsParams<T>& p, int b,
        int& r0, int& c0)
{
    const int cb = b >> 4, q = b & 15;
    r0 = ((cb / p.ncoarse) * kCoarse + (q >> 2)) * kTile;
    c0 = ((cb % p.ncoarse) * kCoarse + (q & 3)) * kTile;
}

// Bin of the fine tile (tu, tv) in that numbering.
static_assert(kCoarse == 4, "fine_bin assumes 4 x 4-tile blocks");
template<typename T>
__device__ __forceinline__ int fine_bin(const EsParams<T>& p, int tu, int tv)
{
    // tu, tv >= 0 (tile indices of in-grid taps): unsigned shifts / masks.
    const unsigned u = (unsigned)tu, v = (unsigned)tv;
    return (int)((((u >> 2) * (unsigned)p.ncoarse + (v >> 2)) << 4) |
            ((u & 3u) << 2) | (v & 3u));
}


// Bucketing kernels ---------------------------------------------------------

template<typename T>
__device__ __forceinline__ T chan_quotient(const T* __restrict__ freq, int c)
{
    return freq[c] / T(kSpeedOfLight);
}

// Tile range of a footprint (grid mode: every tile the support touches;
// degrid: the tile of the first tap) and its super-bin range.
template<typename T, int MODE>
__device__ __forceinline__ void tile_span(const EsParams<T>& p, int u0, int u1,
        int v0, int v1, int& tu0, int& tu1, int& tv0, int& tv1)
{
    const int half = p.G / 2;
    tu0 = (u0 + half) / kTile;
    tv0 = (v0 + half) / kTile;
    tu1 = MODE == MODE_GRID ? (u1 + half) / kTile : tu0;
    tv1 = MODE == MODE_GRID ? (v1 + half) / kTile : tv0;
}

// Counting pass. A workgroup takes kCountChunks consecutive chunks of rows:
// per chunk it counts the records of every super bin (first level, one per
// visibility and super bin its tiles touch) into the chunk's row of the
// super table [chunks][nsbins], and over all its chunks the records of every
// tile into an LDS histogram that is added (global atomics, nonzero bins)
// to its chunk group's row of the group table [groups][nbins] (kGroupChunks
// chunks per group, the granularity k_bucket_fill2 needs). Round 3 wrote a
// [chunks][tiles + super bins] table (68 MB at config 2), read and
// rewritten by the column scan: ~200 MB of bookkeeping per bucketing.
template<typename T, int MODE, int NT>
__global__ __launch_bounds__(NT) void k_bucket_count(EsParams<T> p,
        int64_t num_rows, int num_chan, int64_t chunk, int nc,
        const T* __restrict__ uvw, const T* __restrict__ freq,
        uint32_t* __restrict__ stable, uint32_t* __restrict__ gtable)
{
    __shared__ uint32_t hist[kBinsPerPass + NT];
    __shared__ uint32_t shist[kCountChunks][kMaxSuperBins];
    const int pass_base = blockIdx.y * kBinsPerPass;
    const int nb = min(kBinsPerPass, p.nbins - pass_base);
    const bool supers = blockIdx.y == 0;
    for (int i = threadIdx.x; i < nb; i += NT) hist[i] = 0;
    if (supers)
        for (int i = threadIdx.x; i < kCountChunks * kMaxSuperBins; i += NT)
            (&shist[0][0])[i] = 0;
    __syncthreads();
    // Chunks are ranges of rows; a thread takes a row and its channels
    // (no 64-bit division per visibility, uvw read once per row).
    const int c_first = blockIdx.x * kCountChunks;
#pragma unroll 1
    for (int q = 0; q < kCountChunks; ++q)
    {
        const int64_t r0 = (int64_t)(c_first + q) * chunk;
        const int64_t r1 = min(num_rows, r0 + chunk);
        uint32_t* sh = shist[q];
        // A thread takes rows (not channels: a wave's lanes then fall on
        // different rows and bins; lanes on one row's channels, which share
        // a few tiles, serialised the LDS atomics: count 259 -> 411 us per
        // launch, round 6).
        for (int64_t r = r0 + threadIdx.x; r < r1; r += NT)
        {
            const T u = uvw[3 * r], v = uvw[3 * r + 1], w = uvw[3 * r + 2];
            for (int c = 0; c < num_chan; ++c)
            {
                Footprint<T> f;
                if (!footprint(p, u, v, w, chan_quotient(freq, c), f))
                    continue;
                int tu0, tu1, tv0, tv1;
                tile_span<T, MODE>(p, f.u0, f.u1, f.v0, f.v1, tu0, tu1, tv0,
                        tv1);
                // A support spans at most 2 tiles / super bins per axis;
                // counts outside the span go to this thread's dummy word.
                const int su0 = tu0 >> p.sshift, sv0 = tv0 >> p.sshift;
                const int su1 = tu1 >> p.sshift, sv1 = tv1 >> p.sshift;
                uint32_t* dmy = &hist[kBinsPerPass + threadIdx.x];
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int c2 = 0; c2 < 2; ++c2)
                    {
                        const int b = fine_bin(p, tu0 + a, tv0 + c2) - pass_base;
                        const bool ok = tu0 + a <= tu1 && tv0 + c2 <= tv1 &&
                                b >= 0 && b < nb;
                        atomicAdd(ok ? &hist[b] : dmy, 1u);
                        if (supers)
                        {
                            const bool oks = su0 + a <= su1 && sv0 + c2 <= sv1;
                            atomicAdd(oks ? &sh[(su0 + a) * p.nsuper + sv0 + c2] :
                                    dmy, 1u);
                        }
                    }
            }
        }
    }
    __syncthreads();
    uint32_t* grow = gtable + (size_t)(c_first / kGroupChunks) * p.nbins +
            pass_base;
    for (int i = threadIdx.x; i < nb; i += NT)
    {
        const uint32_t n = hist[i];
        if (n) atomicAdd(&grow[i], n);
    }
    if (supers)
        for (int q = 0; q < kCountChunks && c_first + q < nc; ++q)
        {
            uint32_t* row = stable + (size_t)(c_first + q) * p.nsbins;
            for (int i = threadIdx.x; i < p.nsbins; i += NT)
                row[i] = shist[q][i];
        }
}

// Per bin: exclusive prefix over chunks (in place) and the bin total.
// Block = 16 waves; lane = bin, wave = contiguous range of chunks. MAXPER:
// rows per wave the registers hold (a uniform bound: the group table's 64
// rows at config 2 take 4 loads per thread, the chunk table's up to 1024
// rows 64; one bound for both issued 60 out-of-range loads per thread on
// the group table, 17.5 us per call).
template<int MAXPER>
__device__ __forceinline__ void scan_columns_block(uint32_t* table,
        int num_chunks, int nbins, uint32_t* __restrict__ bin_count, int bx,
        uint32_t (&part)[16][64])
{
    // nbins = columns = the table row length (tile and super-bin counts).
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int b = bx * 64 + lane;
    const int per = (num_chunks + 15) / 16;
    const int c0 = __builtin_amdgcn_readfirstlane(wave * per);
    const int c1 = min(num_chunks, c0 + per);
    // Raw buffer view of the table: lane offset (bin) in one VGPR, chunk
    // offset in an SGPR; lanes past nbins and chunks past c1 address out of
    // range (loads return 0, stores are dropped).
    const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(table,
            0, (int)((size_t)num_chunks * nbins * 4), 0x00020000);
    const uint32_t voff = b < nbins ? (uint32_t)b * 4u : 0xFFFFFFF0u;
    auto soff = [&](int k) -> uint32_t {
        return c0 + k < c1 ? (uint32_t)((c0 + k) * nbins) * 4u : 0x7FFFFFF0u;
    };
    // The wave's column of counts stays in registers between the two
    // passes (the table is read once).
    uint32_t val[MAXPER];
    uint32_t sum = 0;
#pragma unroll
    for (int k = 0; k < MAXPER; ++k)
    {
        val[k] = (uint32_t)__builtin_amdgcn_raw_buffer_load_b32(rs, voff,
                soff(k), 0);
        sum += val[k];
    }
    part[wave][lane] = sum;
    __syncthreads();
    if (wave == 0)
    {
        uint32_t run = 0;
        for (int k = 0; k < 16; ++k)
        {
            const uint32_t t = part[k][lane];
            part[k][lane] = run;
            run += t;
        }
        if (b < nbins) bin_count[b] = run;
    }
    __syncthreads();
    if (b < nbins)
    {
        uint32_t run = part[wave][lane];
#pragma unroll
        for (int k = 0; k < MAXPER; ++k)
        {
            __builtin_amdgcn_raw_buffer_store_b32(run, rs, voff, soff(k), 0);
            run += val[k];
        }
    }
}

// One launch scans two tables: blocks [0, nblk) the first, the rest the
// second, each with the register bound of its row count.
__global__ __launch_bounds__(1024) void k_scan_columns(uint32_t* table,
        int num_chunks, int nbins, uint32_t* __restrict__ bin_count,
        int nblk, uint32_t* table2, int num_chunks2, int nbins2,
        uint32_t* __restrict__ bin_count2)
{
    __shared__ uint32_t part[16][64];
    constexpr int kMaxPer = kMaxChunks / 16;
    static_assert(kMaxChunks % 16 == 0, "chunks split over 16 waves");
    int bx = blockIdx.x;
    if (bx >= nblk)
    {
        table = table2;
        num_chunks = num_chunks2;
        nbins = nbins2;
        bin_count = bin_count2;
        bx -= nblk;
    }
    const int per = (num_chunks + 15) / 16;   // uniform per block
    if (per <= 4)
        scan_columns_block<4>(table, num_chunks, nbins, bin_count, bx, part);
    else if (per <= 16)
        scan_columns_block<16>(table, num_chunks, nbins, bin_count, bx, part);
    else
        scan_columns_block<kMaxPer>(table, num_chunks, nbins, bin_count, bx,
                part);
}

// Exclusive prefix of bin totals and of work items (pieces of <= kPiece
// entries, at least one per bin), the work item -> bin table, and the
// sentinel kNoBin in item_bin past the last item (tile kernels are
// launched for item_capacity work items and the extra ones exit: no host
// round trip for the item count). One block of 1024 threads; rounds of
// 16 consecutive bins per thread, loaded with 16-byte loads.
constexpr uint32_t kNoBin = 0xFFFFFFFFu;

__device__ __forceinline__ void block_scan_1024(uint32_t& a, uint32_t& b,
        uint32_t* s_a, uint32_t* s_b, uint32_t& tot_a, uint32_t& tot_b)
{
    // Inclusive scan of (a, b) over the block; returns exclusive values and
    // the block totals.
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t ia = a, ib = b;
#pragma unroll
    for (int off = 1; off < 64; off <<= 1)
    {
        const uint32_t xa = __shfl_up(ia, off), xb = __shfl_up(ib, off);
        if (lane >= off) { ia += xa; ib += xb; }
    }
    if (lane == 63) { s_a[wave] = ia; s_b[wave] = ib; }
    __syncthreads();
    if (wave == 0)
    {
        uint32_t wa = lane < 16 ? s_a[lane] : 0, wb = lane < 16 ? s_b[lane] : 0;
#pragma unroll
        for (int off = 1; off < 16; off <<= 1)
        {
            const uint32_t xa = __shfl_up(wa, off), xb = __shfl_up(wb, off);
            if (lane >= off) { wa += xa; wb += xb; }
        }
        if (lane < 16) { s_a[16 + lane] = wa; s_b[16 + lane] = wb; }
    }
    __syncthreads();
    const uint32_t pa = wave ? s_a[16 + wave - 1] : 0;
    const uint32_t pb = wave ? s_b[16 + wave - 1] : 0;
    tot_a = s_a[31];
    tot_b = s_b[31];
    a = pa + ia - a;
    b = pb + ib - b;
    __syncthreads();
}

// Run by one 1024-thread block: the extra last block of k_bucket_fill1
// (round 5; it was its own single-block launch, 12.5 us at config 2,
// serial between the column scans and level 1).
struct ScanBinsArgs
{
    uint32_t* bin_start;
    uint32_t* item_start;
    uint32_t* totals;
    uint32_t* item_bin;
    uint32_t item_capacity;
};

__device__ __forceinline__ void scan_bins_block(
        const uint32_t* __restrict__ bin_count, int nbins,
        uint32_t* __restrict__ bin_start, uint32_t* __restrict__ item_start,
        uint32_t* __restrict__ totals, uint32_t* __restrict__ item_bin,
        uint32_t item_capacity)
{
    constexpr int kPer = 8;
    constexpr int kRound = 1024 * kPer;
    __shared__ uint32_t s_a[32], s_b[32];
    // One output array of a round at a time, so that the global stores are
    // coalesced (a thread owns kPer consecutive bins: storing them directly
    // put every lane of a store instruction on its own line). Thread t's
    // values at t * (kPer + 1) + k: the odd stride spreads a wave's LDS
    // writes over all banks.
    __shared__ uint32_t s_stage[1024 * (kPer + 1)];
    auto slot = [](int i) { return (i / kPer) * (kPer + 1) + i % kPer; };
    const int t = threadIdx.x;
    uint32_t carry_c = 0, carry_i = 0;
    for (int base = 0; base < nbins; base += kRound)
    {
        const int nb = min(kRound, nbins - base);
        const int b0 = base + t * kPer;
        uint32_t n[kPer];
        if (b0 + kPer <= nbins)
        {
            const uint4* src = (const uint4*)(bin_count + b0);
#pragma unroll
            for (int k = 0; k < kPer / 4; ++k)
            {
                const uint4 v = src[k];
                n[4 * k] = v.x; n[4 * k + 1] = v.y;
                n[4 * k + 2] = v.z; n[4 * k + 3] = v.w;
            }
        }
        else
        {
#pragma unroll
            for (int k = 0; k < kPer; ++k)
                n[k] = (b0 + k < nbins) ? bin_count[b0 + k] : 0;
        }
        uint32_t cnt = 0, itm = 0;
#pragma unroll
        for (int k = 0; k < kPer; ++k)
        {
            cnt += n[k];
            if (b0 + k < nbins) itm += max(1u, (n[k] + kPiece - 1) / kPiece);
        }
        uint32_t tot_c, tot_i;
        block_scan_1024(cnt, itm, s_a, s_b, tot_c, tot_i);
        // bin_start
        uint32_t run = carry_c + cnt;
#pragma unroll
        for (int k = 0; k < kPer; ++k)
        {
            s_stage[t * (kPer + 1) + k] = run;
            run += n[k];
        }
        __syncthreads();
        for (int i = t; i < nb; i += 1024) bin_start[base + i] = s_stage[slot(i)];
        __syncthreads();
        // item_start
        run = carry_i + itm;
#pragma unroll
        for (int k = 0; k < kPer; ++k)
        {
            s_stage[t * (kPer + 1) + k] = run;
            if (b0 + k < nbins) run += max(1u, (n[k] + kPiece - 1) / kPiece);
        }
        __syncthreads();
        for (int i = t; i < nb; i += 1024) item_start[base + i] = s_stage[slot(i)];
        __syncthreads();
        // item -> bin: the round's first kRound items through LDS (linear),
        // any further ones (bins split into many pieces) stored directly.
        run = itm;   // item offset inside this round
#pragma unroll
        for (int k = 0; k < kPer; ++k)
        {
            const int bb = b0 + k;
            if (bb >= nbins) break;
            const uint32_t ni = max(1u, (n[k] + kPiece - 1) / kPiece);
            for (uint32_t j = 0; j < ni; ++j)
            {
                const uint32_t r = run + j;
                if (r < (uint32_t)kRound)
                    s_stage[slot((int)r)] = (uint32_t)bb;
                else if (carry_i + r < item_capacity)
                    item_bin[carry_i + r] = (uint32_t)bb;
            }
            run += ni;
        }
        __syncthreads();
        const int ni_lds = (int)min(tot_i, (uint32_t)kRound);
        for (int i = t; i < ni_lds; i += 1024)
            if (carry_i + i < item_capacity) item_bin[carry_i + i] = s_stage[slot(i)];
        __syncthreads();
        carry_c += tot_c;
        carry_i += tot_i;
    }
    if (t == 0)
    {
        bin_start[nbins] = carry_c;
        item_start[nbins] = carry_i;
        totals[0] = carry_c;
        totals[1] = carry_i;
    }
    for (uint32_t k = carry_i + t; k < item_capacity; k += 1024)
        item_bin[k] = kNoBin;
}

// One bucketed record as 16-byte stores (records are 16-byte aligned).
template<typename T, int W>
__device__ __forceinline__ void store_rec(T* dst, const T (&rec)[W])
{
    constexpr int kPer = 16 / sizeof(T);
    using V = __attribute__((ext_vector_type(kPer))) T;
#pragma unroll
    for (int k = 0; k < W; k += kPer)
    {
        V x;
#pragma unroll
        for (int j = 0; j < kPer; ++j) x[j] = rec[k + j];
        *(V*)(dst + k) = x;
    }
}

// Barrier for LDS hand-offs only: unlike __syncthreads it does not wait
// for the wave's outstanding global loads and stores (s_waitcnt vmcnt(0)),
// so prefetched loads and the record stores stay in flight across it.
__device__ __forceinline__ void lds_barrier()
{
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "workgroup", "local");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "workgroup", "local");
}

// Exclusive scan of n <= kMaxSuperBins counts (LDS) into off (LDS); returns
// the total. Callers synchronise before reading off or reusing s_wave.
template<int NT>
__device__ __forceinline__ uint32_t block_scan_counts(const uint32_t* cnt,
        uint32_t* off, int n, uint32_t* s_wave)
{
    constexpr int E = (kMaxSuperBins + NT - 1) / NT;
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    uint32_t v[E];
    uint32_t sum = 0;
#pragma unroll
    for (int e = 0; e < E; ++e)
    {
        const int i = t * E + e;
        v[e] = i < n ? cnt[i] : 0u;
        sum += v[e];
    }
    uint32_t inc = sum;
#pragma unroll
    for (int o = 1; o < 64; o <<= 1)
    {
        const uint32_t x = __shfl_up(inc, o);
        if (lane >= o) inc += x;
    }
    if (lane == 63) s_wave[wave] = inc;
    lds_barrier();
    uint32_t before = 0, total = 0;
#pragma unroll
    for (int w = 0; w < NT / 64; ++w)
    {
        const uint32_t x = s_wave[w];
        before += w < wave ? x : 0u;
        total += x;
    }
    uint32_t run = before + inc - sum;
#pragma unroll
    for (int e = 0; e < E; ++e)
    {
        const int i = t * E + e;
        if (i < n) off[i] = run;
        run += v[e];
    }
    return total;
}

// 16-byte vector copy of one record.
template<typename T, int W>
__device__ __forceinline__ void copy_rec(T* dst, const T* src)
{
    constexpr int kPer = 16 / sizeof(T);
    using V = __attribute__((ext_vector_type(kPer))) T;
#pragma unroll
    for (int k = 0; k < W; k += kPer) *(V*)(dst + k) = *(const V*)(src + k);
}

// Visibilities per thread per batch of the first level: 3 records of 16
// bytes (1 of 32 or 64) per thread, so that the LDS stage of a 1024-thread
// block stays below 80 KiB and two blocks share a CU (one block's loads
// overlap the other's sort and stores).
constexpr int kFill1Bytes = 48;
template<typename T, int W>
struct Fill1Shape
{
    static constexpr int K = (kFill1Bytes / (W * (int)sizeof(T))) > 0 ?
            kFill1Bytes / (W * (int)sizeof(T)) : 1;
};

// First bucketing level: the chunk's records by super bin. A block walks
// its chunk in batches of NT * K visibilities; each batch is counting-
// sorted by super bin in LDS (ranks from LDS atomics, an exclusive scan of
// the batch counts) and then stored in LDS order, so the records of one
// super bin leave as one contiguous run of ~NT * K / nsbins records (full
// cache lines) instead of one 16-byte store per record into a random bin.
// Record layouts as k_bucket_fill's were: see es_kernels.h. Positions in
// a super bin follow the chunk order (scanned count-table columns), which
// lets k_bucket_fill2 find the records of any chunk range.
// One 1024-thread block per CU (VGPR budget 128; two blocks need <= 64
// VGPRs and spill).
template<typename T, int MODE, bool DO_W, int NT>
__global__ __launch_bounds__(NT) __attribute__((amdgpu_waves_per_eu(
        NT / 256))) void k_bucket_fill1(EsParams<T> p,
        int64_t num_rows, int num_chan, int64_t chunk, const T* __restrict__ uvw,
        const T* __restrict__ freq, const T* __restrict__ vis,
        const T* __restrict__ weight, const uint32_t* __restrict__ stable,
        const uint32_t* __restrict__ bin_count, uint32_t* __restrict__ sb_start,
        T* __restrict__ recs1, ScanBinsArgs sba)
{
    static_assert(NT == 1024, "the extra block runs scan_bins_block");
    if (blockIdx.x == gridDim.x - 1)
    {
        // Tile-bin / work-item prefix for level 2 and the tile kernels: it
        // needs only the column scans, so it runs beside level 1.
        scan_bins_block(bin_count, p.nbins, sba.bin_start, sba.item_start,
                sba.totals, sba.item_bin, sba.item_capacity);
        return;
    }
    constexpr int kWords = Rec<T, MODE, DO_W>::kWords;
    constexpr int K = Fill1Shape<T, kWords>::K;
    constexpr int kBatch = NT * K;
    constexpr int kCap = kBatch + kBatch / 8;   // staged records per round
    __shared__ uint32_t cursor[kMaxSuperBins];
    __shared__ uint32_t lcnt[kMaxSuperBins];
    __shared__ uint32_t loff[kMaxSuperBins];
    __shared__ uint32_t s_wave[NT / 64];
    __shared__ __attribute__((aligned(16))) T stage[kCap * kWords];
    __shared__ uint16_t stage_sb[kCap];
    const int t = threadIdx.x;
    const int nsb = p.nsbins;
    // Super-bin starts (scan of the totals; block 0 stores them for
    // k_bucket_fill2) + this chunk's offset in each.
    const uint32_t n_sb = block_scan_counts<NT>(bin_count + p.nbins, loff,
            nsb, s_wave);
    __syncthreads();
    const uint32_t* row = stable + (size_t)blockIdx.x * p.nsbins;
    for (int i = t; i < nsb; i += NT)
    {
        cursor[i] = loff[i] + row[i];
        lcnt[i] = 0;
        if (blockIdx.x == 0) sb_start[i] = loff[i];
    }
    if (blockIdx.x == 0 && t == 0) sb_start[nsb] = n_sb;
    __syncthreads();
    const int64_t r0 = (int64_t)blockIdx.x * chunk;
    const int64_t r1 = min(num_rows, r0 + chunk);
    const uint32_t nvis = r1 > r0 ? (uint32_t)((r1 - r0) * num_chan) : 0u;
    // The chunk's inputs from scalar base pointers (32-bit offsets); row of
    // a visibility by a multiply-high with a one-step correction.
    const T* __restrict__ uvw_c = uvw + 3 * r0;
    const T* __restrict__ vis_c = MODE == MODE_GRID ? vis + 2 * r0 * num_chan : vis;
    const T* __restrict__ wt_c = MODE == MODE_GRID ? weight + r0 * num_chan : weight;
    const uint32_t nch = (uint32_t)num_chan;
    const uint32_t magic = nch > 1 ? (uint32_t)(0x100000000ull / nch) : 0u;
    // NT % C == 0: every visibility of this thread (chunk-local index
    // b0 + k NT + t, b0 a multiple of NT) has channel t % C, so its channel
    // quotient is formed once.
    const bool chan_fixed = num_chan > 0 && NT % num_chan == 0;
    const T iwl_t = chan_fixed ? chan_quotient(freq, t % num_chan) : T(0);
    // The inputs of a batch are loaded one batch ahead (K visibilities per
    // thread; consecutive lanes = consecutive visibilities, so the vis /
    // weight loads are coalesced and a row's uvw is shared by its
    // channels): their latency overlaps the sort and stores of the batch
    // before (the barriers below are LDS-only).
    T in_u[K], in_v[K], in_w[K], in_f[K], in_re[K], in_im[K], in_wt[K];
    auto load_batch = [&](uint32_t b0) {
#pragma unroll
        for (int k = 0; k < K; ++k)
        {
            const uint32_t li = min(b0 + (uint32_t)(k * NT + t), nvis - 1);
            uint32_t rl = li;
            if (nch > 1)
            {
                rl = __umulhi(li, magic);
                if (li - rl * nch >= nch) ++rl;
            }
            const uint32_t c = li - rl * nch;
            in_u[k] = uvw_c[3 * rl];
            in_v[k] = uvw_c[3 * rl + 1];
            in_w[k] = uvw_c[3 * rl + 2];
            in_f[k] = chan_fixed ? iwl_t : chan_quotient(freq, (int)c);
            if constexpr (MODE == MODE_GRID)
            {
                in_re[k] = vis_c[2 * li];
                in_im[k] = vis_c[2 * li + 1];
                in_wt[k] = wt_c[li];
            }
        }
    };
    if (nvis) load_batch(0);
    for (uint32_t base = 0; base < nvis; base += kBatch)
    {
        T rec[K][kWords];
        uint32_t rank[K][2];
        // Super bins of entry k: first sbase, + 1 (v) if bit 16, + nsuper
        // (u) if bit 17; bit 18 = entry present.
        uint32_t span[K];
#pragma unroll
        for (int k = 0; k < K; ++k)
        {
            span[k] = 0;
            rank[k][0] = rank[k][1] = 0;
            const uint32_t li = base + (uint32_t)(k * NT + t);
            if (li >= nvis) continue;
            Footprint<T> f;
            if (!footprint(p, in_u[k], in_v[k], in_w[k], in_f[k], f)) continue;
            rec[k][0] = f.pu;
            rec[k][1] = f.pv;
            if constexpr (MODE == MODE_GRID)
            {
                // kernels.cu:163-167: weight, then conjugate for w < 0.
                const T wt = in_wt[k];
                rec[k][2] = in_re[k] * wt;
                T vim = in_im[k] * wt;
                vim *= f.flip;
                rec[k][3] = vim;
                if constexpr (DO_W && kWords == 8)
                {
                    rec[k][4] = f.kw;
                    rec[k][5] = rec[k][6] = rec[k][7] = T(0);
                }
            }
            else
            {
                rec[k][2] = copysign(f.kw, f.flip);
                rec[k][3] = idx_bits(T(0),
                        (uint64_t)(r0 * num_chan) + (uint64_t)li);
            }
            int tu0, tu1, tv0, tv1;
            tile_span<T, MODE>(p, f.u0, f.u1, f.v0, f.v1, tu0, tu1, tv0, tv1);
            const int su0 = tu0 >> p.sshift, sv0 = tv0 >> p.sshift;
            // A support (<= 64 cells) spans at most 2 super bins per axis.
            span[k] = (uint32_t)(su0 * p.nsuper + sv0) | (1u << 18) |
                    ((uint32_t)((tv1 >> p.sshift) - sv0) << 16) |
                    ((uint32_t)((tu1 >> p.sshift) - su0) << 17);
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                {
                    if ((a && !(span[k] & (1u << 17))) ||
                            (b && !(span[k] & (1u << 16)))) continue;
                    const int sb = (int)(span[k] & 0xFFFFu) + a * p.nsuper + b;
                    const uint32_t q = atomicAdd(&lcnt[sb], 1u);
                    rank[k][a] |= q << (16 * b);
                }
        }
        if (base + kBatch < nvis) load_batch(base + kBatch);
        lds_barrier();
        const uint32_t total = block_scan_counts<NT>(lcnt, loff, nsb, s_wave);
        lds_barrier();
        // Rounds of kCap staged records (one round unless many visibilities
        // of the batch straddle super bins).
        for (uint32_t s0 = 0; s0 < total; s0 += kCap)
        {
#pragma unroll
            for (int k = 0; k < K; ++k)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                    {
                        if (!(span[k] & (1u << 18)) ||
                                (a && !(span[k] & (1u << 17))) ||
                                (b && !(span[k] & (1u << 16)))) continue;
                        const int sb = (int)(span[k] & 0xFFFFu) + a * p.nsuper + b;
                        const uint32_t slot = loff[sb] +
                                ((rank[k][a] >> (16 * b)) & 0xFFFFu) - s0;
                        if (slot >= (uint32_t)kCap) continue;
                        store_rec<T, kWords>(stage + slot * kWords, rec[k]);
                        stage_sb[slot] = (uint16_t)sb;
                    }
            lds_barrier();
            const uint32_t n = min((uint32_t)kCap, total - s0);
            for (uint32_t j = t; j < n; j += NT)
            {
                const int sb = stage_sb[j];
                const uint32_t pos = cursor[sb] + (s0 + j - loff[sb]);
                copy_rec<T, kWords>(recs1 + (size_t)pos * kWords,
                        stage + j * kWords);
            }
            lds_barrier();
        }
        for (int i = t; i < nsb; i += NT)
        {
            cursor[i] += lcnt[i];
            lcnt[i] = 0;
        }
        lds_barrier();
    }
}

// Second level: the records of super bin blockIdx.y that come from chunks
// [c0, c0 + gc) (contiguous in recs1) into their tiles. A record is
// written to every tile of this super bin its support touches (grid) or
// the tile of its first tap (degrid); tile f's records from these chunks
// occupy [bin_start[f] + table[c0][f], ...), a window of a few hundred
// bytes per tile that the block fills while it stays in L2.
template<typename T, int MODE, bool DO_W>
__global__ __launch_bounds__(256) void k_bucket_fill2(EsParams<T> p, int nc,
        const uint32_t* __restrict__ stable,
        uint32_t* __restrict__ gtable,
        const uint32_t* __restrict__ bin_count,
        const uint32_t* __restrict__ bin_start,
        const uint32_t* __restrict__ sb_start, const T* __restrict__ recs1,
        T* __restrict__ recs)
{
    constexpr int kWords = Rec<T, MODE, DO_W>::kWords;
    __shared__ uint32_t cur[kMaxSuperTiles];
    const int t = threadIdx.x, sb = blockIdx.y;
    const int c0 = blockIdx.x * kGroupChunks;
    if (c0 >= nc) return;
    const int c1 = min(nc, c0 + kGroupChunks);
    const int S = 1 << p.sshift;
    const int su = sb / p.nsuper, sv = sb - su * p.nsuper;
    const int tu_base = su << p.sshift, tv_base = sv << p.sshift;
    const uint32_t* col = stable + sb;
    const uint32_t sbs = sb_start[sb];
    const uint32_t e0 = sbs + col[(size_t)c0 * p.nsbins];
    const uint32_t e1 = c1 < nc ? sbs + col[(size_t)c1 * p.nsbins] :
            sb_start[sb + 1];
    // Four records per thread in flight (loads issued before the LDS
    // atomics and stores of the first). Gridding: the first round's loads
    // are issued before the tile cursors are set up, so that the two
    // overlap (108 -> 102 us 2-D, 210 -> 191 us 3-D at config 2; the degrid
    // records measured 84 -> 90 us that way).
    constexpr bool kEarly = MODE == MODE_GRID;
    constexpr int kIn = 4;
    T rec[kIn][kWords];
    auto load = [&](uint32_t e) {
#pragma unroll
        for (int q = 0; q < kIn; ++q)
            if (e + q * 256 < e1)
                copy_rec<T, kWords>(rec[q],
                        recs1 + (size_t)(e + q * 256) * kWords);
    };
    if (kEarly) load(e0 + t);
    for (int j = t; j < S * S; j += 256)
    {
        const int tu = tu_base + (j >> p.sshift), tv = tv_base + (j & (S - 1));
        if (tu < p.ntiles && tv < p.ntiles)
        {
            const int f = fine_bin(p, tu, tv);
            uint32_t* g = gtable + (size_t)blockIdx.x * p.nbins + f;
            cur[j] = bin_start[f] + *g;
            // This block is the entry's only reader: leave the table zeroed
            // for the next bucketing's atomic counts (no memset per call).
            *g = 0u;
        }
    }
    __syncthreads();
    for (uint32_t e = e0 + t; e < e1; e += 256 * kIn)
    {
        if (!kEarly || e != e0 + t) load(e);
        // All cursor atomics of the kIn records first, then the stores: a
        // store right behind its atomic waits for the LDS round trip, and
        // the next record's atomic behind that store (config 3: level-2
        // stores 5.6 of 7.1 ms per call with the interleaved form).
        uint32_t pos[kIn][2][2];
        bool put[kIn][2][2];
#pragma unroll
        for (int q = 0; q < kIn; ++q)
        {
            const bool in = e + q * 256 < e1;
            int u0, u1, v0, v1, tu0 = 0, tu1 = -1, tv0 = 0, tv1 = -1;
            if (in)
            {
                tap_range(p, rec[q][0], rec[q][1], u0, u1, v0, v1);
                tile_span<T, MODE>(p, u0, u1, v0, v1, tu0, tu1, tv0, tv1);
                tu0 = max(tu0, tu_base); tu1 = min(tu1, tu_base + S - 1);
                tv0 = max(tv0, tv_base); tv1 = min(tv1, tv_base + S - 1);
            }
            // A support spans at most 2 tiles per axis.
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                {
                    const int tu = tu0 + a, tv = tv0 + b;
                    put[q][a][b] = tu <= tu1 && tv <= tv1;
                    pos[q][a][b] = 0;
                    if (put[q][a][b])
                        pos[q][a][b] = atomicAdd(&cur[((tu - tu_base) <<
                                p.sshift) | (tv - tv_base)], 1u);
                }
        }
#pragma unroll
        for (int q = 0; q < kIn; ++q)
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                    if (put[q][a][b])
                        store_rec<T, kWords>(recs + (size_t)pos[q][a][b] *
                                kWords, rec[q]);
    }
}


// Second level, staged form for blocks of many records (C >> 1: ~16 k
// records per block at config 3; chosen on the host from the average,
// launch_fill). Rounds of kF2Round records:
// each is counting-sorted by tile in LDS (ranks from LDS atomics, a scan of
// the round's tile counts) and leaves as one contiguous run per tile
// (consecutive threads, consecutive addresses) instead of one 16-byte
// store per record (round 5: at config 3 the scattered stores were 5.6 of
// the level's 7.1 ms per call; staged 15.13 -> 14.24 ms bucketing per
// call; at config 2's ~600 records per block the direct form is faster,
// 0.288 vs 0.297 ms).
constexpr int kF2In = 4;                       // records per thread per round
constexpr int kF2Round = 256 * kF2In;
constexpr int kF2Cap = kF2Round + kF2Round / 4;   // staged outputs per pass

template<typename T, int MODE, bool DO_W>
size_t fill2_lds_bytes(int ntile)
{
    constexpr int kWords = Rec<T, MODE, DO_W>::kWords;
    return (size_t)kF2Cap * kWords * sizeof(T) + (size_t)kF2Cap * 4 +
            3 * (size_t)ntile * 4;
}

template<typename T, int MODE, bool DO_W>
__global__ __launch_bounds__(256) void k_bucket_fill2_staged(EsParams<T> p, int nc,
        const uint32_t* __restrict__ stable,
        uint32_t* __restrict__ gtable,
        const uint32_t* __restrict__ bin_count,
        const uint32_t* __restrict__ bin_start,
        const uint32_t* __restrict__ sb_start, const T* __restrict__ recs1,
        T* __restrict__ recs)
{
    constexpr int kWords = Rec<T, MODE, DO_W>::kWords;
    extern __shared__ __attribute__((aligned(16))) unsigned char f2_lds[];
    const int t = threadIdx.x, sb = blockIdx.y;
    const int c0 = blockIdx.x * kGroupChunks;
    if (c0 >= nc) return;
    const int c1 = min(nc, c0 + kGroupChunks);
    const int S = 1 << p.sshift, ntile = S * S;
    T* stage = (T*)f2_lds;                                     // [kF2Cap][kWords]
    uint32_t* stage_j = (uint32_t*)(stage + (size_t)kF2Cap * kWords);
    uint32_t* cur = stage_j + kF2Cap;                          // [ntile]
    uint32_t* lcnt = cur + ntile;
    uint32_t* loff = lcnt + ntile;
    __shared__ uint32_t s_wave[4];
    const int su = sb / p.nsuper, sv = sb - su * p.nsuper;
    const int tu_base = su << p.sshift, tv_base = sv << p.sshift;
    const uint32_t* col = stable + sb;
    const uint32_t sbs = sb_start[sb];
    const uint32_t e0 = sbs + col[(size_t)c0 * p.nsbins];
    const uint32_t e1 = c1 < nc ? sbs + col[(size_t)c1 * p.nsbins] :
            sb_start[sb + 1];
    T rec[kF2In][kWords];
    auto load = [&](uint32_t rb) {
#pragma unroll
        for (int q = 0; q < kF2In; ++q)
            if (rb + t + q * 256 < e1)
                copy_rec<T, kWords>(rec[q],
                        recs1 + (size_t)(rb + t + q * 256) * kWords);
    };
    load(e0);
    for (int j = t; j < ntile; j += 256)
    {
        const int tu = tu_base + (j >> p.sshift), tv = tv_base + (j & (S - 1));
        lcnt[j] = 0;
        if (tu < p.ntiles && tv < p.ntiles)
        {
            const int f = fine_bin(p, tu, tv);
            uint32_t* g = gtable + (size_t)blockIdx.x * p.nbins + f;
            cur[j] = bin_start[f] + *g;
            // This block is the entry's only reader: leave the table zeroed
            // for the next bucketing's atomic counts (no memset per call).
            *g = 0u;
        }
    }
    __syncthreads();
    for (uint32_t rb = e0; rb < e1; rb += kF2Round)
    {
        if (rb != e0) load(rb);
        // Tile slots of this round's records (a support spans at most two
        // tiles per axis) and their ranks in the round's tile runs.
        uint32_t rank[kF2In][2][2];
        int jj[kF2In][2][2];
#pragma unroll
        for (int q = 0; q < kF2In; ++q)
        {
            const bool in = rb + t + q * 256 < e1;
            int u0, u1, v0, v1, tu0 = 0, tu1 = -1, tv0 = 0, tv1 = -1;
            if (in)
            {
                tap_range(p, rec[q][0], rec[q][1], u0, u1, v0, v1);
                tile_span<T, MODE>(p, u0, u1, v0, v1, tu0, tu1, tv0, tv1);
                tu0 = max(tu0, tu_base); tu1 = min(tu1, tu_base + S - 1);
                tv0 = max(tv0, tv_base); tv1 = min(tv1, tv_base + S - 1);
            }
#pragma unroll
            for (int a = 0; a < 2; ++a)
#pragma unroll
                for (int b = 0; b < 2; ++b)
                {
                    const int tu = tu0 + a, tv = tv0 + b;
                    jj[q][a][b] = -1;
                    rank[q][a][b] = 0;
                    if (tu <= tu1 && tv <= tv1)
                    {
                        const int j = ((tu - tu_base) << p.sshift) |
                                (tv - tv_base);
                        jj[q][a][b] = j;
                        rank[q][a][b] = atomicAdd(&lcnt[j], 1u);
                    }
                }
        }
        __syncthreads();
        // Exclusive scan of the round's tile counts (ntile <= 4096).
        uint32_t total;
        {
            constexpr int E = kMaxSuperTiles / 256;
            const int lane = t & 63, wave = t >> 6;
            uint32_t v[E];
            uint32_t sum = 0;
#pragma unroll
            for (int k = 0; k < E; ++k)
            {
                const int i = t * E + k;
                v[k] = i < ntile ? lcnt[i] : 0u;
                sum += v[k];
            }
            uint32_t inc = sum;
#pragma unroll
            for (int o = 1; o < 64; o <<= 1)
            {
                const uint32_t x = __shfl_up(inc, o);
                if (lane >= o) inc += x;
            }
            if (lane == 63) s_wave[wave] = inc;
            __syncthreads();
            uint32_t before = 0;
            total = 0;
#pragma unroll
            for (int w = 0; w < 4; ++w)
            {
                const uint32_t x = s_wave[w];
                before += w < wave ? x : 0u;
                total += x;
            }
            uint32_t run = before + inc - sum;
#pragma unroll
            for (int k = 0; k < E; ++k)
            {
                const int i = t * E + k;
                if (i < ntile) loff[i] = run;
                run += v[k];
            }
        }
        __syncthreads();
        for (uint32_t s0 = 0; s0 < total; s0 += kF2Cap)
        {
#pragma unroll
            for (int q = 0; q < kF2In; ++q)
#pragma unroll
                for (int a = 0; a < 2; ++a)
#pragma unroll
                    for (int b = 0; b < 2; ++b)
                    {
                        const int j = jj[q][a][b];
                        if (j < 0) continue;
                        const uint32_t slot = loff[j] + rank[q][a][b] - s0;
                        if (slot >= (uint32_t)kF2Cap) continue;
                        store_rec<T, kWords>(stage + (size_t)slot * kWords,
                                rec[q]);
                        stage_j[slot] = (uint32_t)j;
                    }
            __syncthreads();
            const uint32_t n = min((uint32_t)kF2Cap, total - s0);
            for (uint32_t i = t; i < n; i += 256)
            {
                const uint32_t j = stage_j[i];
                const uint32_t pos = cur[j] + (s0 + i - loff[j]);
                copy_rec<T, kWords>(recs + (size_t)pos * kWords,
                        stage + (size_t)i * kWords);
            }
            __syncthreads();
        }
        for (int j = t; j < ntile; j += 256)
        {
            cur[j] += lcnt[j];
            lcnt[j] = 0;
        }
        __syncthreads();
    }
}


// Zero the grid cells of tiles that several work items share.
template<typename T>
__global__ __launch_bounds__(kThreads) void k_zero_shared_tiles(
        EsParams<T> p, const uint32_t* __restrict__ item_start, T* grid)
{
    const int b = blockIdx.x;
    if (item_start[b + 1] - item_start[b] <= 1) return;
    int r0, c0;
    tile_origin(p, b, r0, c0);
    const int G = p.G;
    const int nr = min(kTile, G - r0), nc = min(kTile, G - c0);
    for (int k = threadIdx.x; k < nr * nc * 2; k += kThreads)
    {
        const int r = k / (2 * nc), c = k - r * 2 * nc;
        grid[((size_t)(r0 + r) * G + c0) * 2 + c] = T(0);
    }
}

// Wave-uniform broadcast of lane j's value (v_readlane -> SGPR).
__device__ __forceinline__ int lane_bcast(int x, int j)
{
    return __builtin_amdgcn_readlane(x, j);
}
__device__ __forceinline__ float lane_bcast(float x, int j)
{
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(x), j));
}
__device__ __forceinline__ double lane_bcast(double x, int j)
{
    const long long b = __double_as_longlong(x);
    const int lo = __builtin_amdgcn_readlane((int)(b & 0xffffffffll), j);
    const int hi = __builtin_amdgcn_readlane((int)(b >> 32), j);
    return __longlong_as_double(((long long)hi << 32) | (unsigned int)lo);
}

// One batch of up to 64 bucketed records, one per lane, with the per-entry
// tap window (relative to the tile) packed for wave-uniform decoding:
//   win = lo_u | (hi_u + 1) << 8 | lo_v << 16 | (hi_v + 1) << 24
//   org = (u0 - tu0 + 256) | (v0 - tv0 + 256) << 16
// where lo/hi are tap offsets from the entry's first tap u0 / v0 that lie
// inside [tile, tile + kTile) (the whole window in gather mode).
template<typename T>
struct Batch
{
    T pu, pv, a, b, kw;
    int u0, v0;
    int win, org;
    uint64_t wide;   // entries with more than 8 taps on an axis
    int cnt;
};

template<typename T, bool DO_W, int WORDS>
__device__ __forceinline__ void load_batch(const EsParams<T>& p,
        const T* __restrict__ recs, uint32_t base, uint32_t end, int lane,
        int tu0, int tv0, int clip_rows, Batch<T>& bt)
{
    bt.cnt = (int)min(64u, end - base);
    bt.pu = T(0);
    bt.pv = T(0);
    bt.a = T(0);
    bt.b = T(0);
    bt.kw = T(1);
    if (lane < bt.cnt)
    {
        const T* r = recs + (size_t)(base + lane) * WORDS;
        bt.pu = r[0];
        bt.pv = r[1];
        bt.a = r[2];
        bt.b = r[3];
        if (DO_W) (void)plane_tap(p, r[4], bt.kw);   // 0 off this plane
    }
    int u1, v1;
    tap_range(p, bt.pu, bt.pv, bt.u0, u1, bt.v0, v1);
    const int lo_u = max(bt.u0, tu0) - bt.u0;
    const int hi_u = min(u1, tu0 + clip_rows - 1) - bt.u0;
    const int lo_v = max(bt.v0, tv0) - bt.v0;
    const int hi_v = min(v1, tv0 + clip_rows - 1) - bt.v0;
    bt.win = lo_u | ((hi_u + 1) << 8) | (lo_v << 16) | ((hi_v + 1) << 24);
    bt.org = (bt.u0 - tu0 + 256) | ((bt.v0 - tv0 + 256) << 16);
    bt.wide = __ballot(lane < bt.cnt && (u1 - bt.u0 > 7 || v1 - bt.v0 > 7));
}

// Cooperative ES taps for entries g..g+3 of a batch: lane L evaluates tap
// (L & 7) of axis (L >> 3) & 1 (0 = u, 1 = v) of entry g + (L >> 4), with
// exactly the reference's arithmetic for grid coordinate u0 + t.
template<typename T>
__device__ __forceinline__ T group_taps(const EsParams<T>& p,
        const Batch<T>& bt, int g, int lane, T inv_hs)
{
    // (A shuffle returns the SOURCE lane's value, so fetch both axes and
    // select on the reading side.)
    const int jsel = g + (lane >> 4);
    const bool axis_v = (lane >> 3) & 1;
    const T pu = __shfl(bt.pu, jsel), pv = __shfl(bt.pv, jsel);
    const int u0 = __shfl(bt.u0, jsel), v0 = __shfl(bt.v0, jsel);
    const T ps = axis_v ? pv : pu;
    const int ss = axis_v ? v0 : u0;
    return es_tap(p.beta, ((T)(ss + (lane & 7)) - ps) * inv_hs);
}

// Grid mode: one workgroup per work item. The tile is accumulated in LDS
// (planar re / im, row stride 72: the 8x8 tap block of a wave is
// bank-conflict free) and written to HBM once.
// Per wave: records are loaded 64 at a time (one per lane, coalesced); the
// 16 taps of four entries are evaluated by the 64 lanes together, then each
// entry is applied by the whole wave, lane = (du, dv) tap, two ds_add_f32.
template<typename T, bool DO_W>
__global__ __launch_bounds__(kThreads) void k_scatter(EsParams<T> p,
        const T* __restrict__ recs, const uint32_t* __restrict__ bin_start,
        const uint32_t* __restrict__ item_start,
        const uint32_t* __restrict__ item_bin, T* __restrict__ grid,
        int accumulate)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int S = kScatterStride;
    constexpr int kWords = Rec<T, MODE_GRID, DO_W>::kWords;
    T* s_re = (T*)smem;
    T* s_im = s_re + kTile * S;
    for (int k = threadIdx.x; k < kTile * S; k += kThreads)
    {
        s_re[k] = T(0);
        s_im[k] = T(0);
    }
    const uint32_t item = blockIdx.x;
    if (item_bin[item] == kNoBin) return;   // past the last work item
    const int b = (int)item_bin[item];
    const uint32_t piece = item - item_start[b];
    const uint32_t npieces = item_start[b + 1] - item_start[b];
    const uint32_t e0 = bin_start[b] + piece * kPiece;
    const uint32_t e1 = min(bin_start[b + 1], e0 + kPiece);
    if (accumulate && e0 == e1) return;     // nothing to add
    const int half = p.G / 2;
    int r0, c0;
    tile_origin(p, b, r0, c0);
    if (r0 >= p.G || c0 >= p.G) return;    // phantom tile
    const int tu0 = r0 - half, tv0 = c0 - half;   // signed coords of tile
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int du = lane >> 3, dv = lane & 7;
    const int lane_off = du * S + dv;
    const int lane_par = (du + dv) & 1;
    const T inv_hs = T(1) / (T(p.support) / T(2));
    for (uint32_t base = e0 + wave * 64; base < e1; base += kWaves * 64)
    {
        Batch<T> bt;
        load_batch<T, DO_W, kWords>(p, recs, base, e1, lane, tu0, tv0, kTile,
                bt);
        for (int g = 0; g < bt.cnt; g += 4)
        {
            const T es = group_taps(p, bt, g, lane, inv_hs);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
            {
                const int j = g + jj;
                if (j >= bt.cnt) break;
                const T ku = __shfl(es, (jj << 4) | du);
                const T kv = __shfl(es, (jj << 4) | 8 | dv);
                const T vre = lane_bcast(bt.a, j), vim = lane_bcast(bt.b, j);
                const T kw = DO_W ? lane_bcast(bt.kw, j) : T(1);
                if ((bt.wide >> j) & 1ull)
                {
                    // Rare: a tap exactly on +-W/2 gives W+1 taps on an
                    // axis. Generic per-lane loop over the tile window.
                    const T pu = lane_bcast(bt.pu, j), pv = lane_bcast(bt.pv, j);
                    int u0, u1, v0, v1;
                    tap_range(p, pu, pv, u0, u1, v0, v1);
                    u0 = max(u0, tu0);
                    u1 = min(u1, tu0 + kTile - 1);
                    v0 = max(v0, tv0);
                    v1 = min(v1, tv0 + kTile - 1);
                    for (int ub = u0; ub <= u1; ub += 8)
                        for (int vb = v0; vb <= v1; vb += 8)
                        {
                            const int u = ub + du, v = vb + dv;
                            if (u <= u1 && v <= v1)
                            {
                                const T k = tap_weight(p, u, v, pu, pv, kw);
                                const int a = (u - tu0) * S + (v - tv0);
                                atomicAdd(&s_re[a], vre * k);
                                atomicAdd(&s_im[a], vim * k);
                            }
                        }
                    continue;
                }
                const int win = lane_bcast(bt.win, j);
                const int org = lane_bcast(bt.org, j);
                const bool act = du >= (win & 255) && du < ((win >> 8) & 255) &&
                        dv >= ((win >> 16) & 255) && dv < (win >> 24);
                T k = ku * kv;
                if (DO_W) k *= kw;
                if ((lane_par + org + (org >> 16)) & 1) k = -k;
                if (act)
                {
                    const int a = lane_off + ((org & 0xffff) - 256) * S +
                            ((org >> 16) - 256);
                    atomicAdd(&s_re[a], vre * k);
                    atomicAdd(&s_im[a], vim * k);
                }
            }
        }
    }
    __syncthreads();

    const int nr = min(kTile, p.G - r0), nc = min(kTile, p.G - c0);
    if (npieces == 1 && accumulate)
    {
        // Batched call: this tile's only work item of the batch adds to
        // the grid (no other writer during this launch).
        for (int k = threadIdx.x; k < kTile * 2 * kTile; k += kThreads)
        {
            const int r = k / (2 * kTile), f = k - r * 2 * kTile;
            const int c = f >> 1;
            if (r >= nr || c >= nc) continue;
            const T val = (f & 1) ? s_im[r * S + c] : s_re[r * S + c];
            grid[((size_t)(r0 + r) * p.G + c0) * 2 + f] += val;
        }
    }
    else if (npieces == 1)
    {
        // Plain stores: 2 cells (float) / 1 cell (double) = 16 B per lane.
        constexpr int kCells = sizeof(T) == 4 ? 2 : 1;
        constexpr int kPerRow = kTile / kCells;
        for (int k = threadIdx.x; k < kTile * kPerRow; k += kThreads)
        {
            const int r = k / kPerRow, c = (k - r * kPerRow) * kCells;
            if (r >= nr || c >= nc) continue;
            T* dst = grid + ((size_t)(r0 + r) * p.G + c0 + c) * 2;
            if constexpr (kCells == 2)
            {
                float4 v;
                v.x = (float)s_re[r * S + c];
                v.y = (float)s_im[r * S + c];
                v.z = (float)s_re[r * S + c + 1];
                v.w = (float)s_im[r * S + c + 1];
                *(float4*)dst = v;
            }
            else
            {
                double2 v;
                v.x = (double)s_re[r * S + c];
                v.y = (double)s_im[r * S + c];
                *(double2*)dst = v;
            }
        }
    }
    else
    {
        // Shared tile: 256 contiguous bytes of f32 adds per wave-instruction.
        for (int k = threadIdx.x; k < kTile * 2 * kTile; k += kThreads)
        {
            const int r = k / (2 * kTile), f = k - r * 2 * kTile;
            const int c = f >> 1;
            if (r >= nr || c >= nc) continue;
            const T val = (f & 1) ? s_im[r * S + c] : s_re[r * S + c];
            if (val != T(0))
                unsafeAtomicAdd(grid + ((size_t)(r0 + r) * p.G + c0) * 2 + f,
                        val);
        }
    }
}

// Atomic-free visit pool of one chunk (tap-table kernels). Phase 1, before
// a barrier: each wave ballots its entries per sub-tile, keeps for every
// hit the entry's rank inside the ballot, and lane st publishes the wave's
// count for sub-tile st. Phase 2, after it: every wave derives the pool
// layout itself (sub-tile-major, wave-minor) with a 32-lane scan, so no
// LDS atomics and no serial prefix stand between the barriers.
template<int kNS>
struct PoolCounts
{
    uint32_t c[4][kNS];
};

template<int kSub>
__device__ __forceinline__ void pool_count(PoolCounts<kSub * kSub>& pc,
        int lane, int wave, int wlo_r, int whi_r, int wlo_c, int whi_c,
        int sub[4], int rank[4])
{
    int nh = 0;
    uint32_t my_cnt = 0;
#pragma unroll
    for (int st = 0; st < kSub * kSub; ++st)
    {
        const int sr = st / kSub, sc = st % kSub;
        const bool hit = sr >= wlo_r && sr <= whi_r && sc >= wlo_c &&
                sc <= whi_c;
        const uint64_t m = __ballot(hit);
        if (lane == st) my_cnt = (uint32_t)__popcll(m);
        if (hit && nh < 4)
        {
            sub[nh] = st;
            rank[nh] = (int)__popcll(m & ((1ull << lane) - 1ull));
            ++nh;
        }
    }
    for (int k = nh; k < 4; ++k) sub[k] = -1;
    if (lane < kSub * kSub) pc.c[wave][lane] = my_cnt;
}

// Lane L < kNS receives sub-tile L's pool begin and size, and the begin
// of this wave's part of it.
template<int kNS>
__device__ __forceinline__ void pool_layout(const PoolCounts<kNS>& pc,
        int lane, int wave, int& beg, int& tot, int& base)
{
    int t = 0, pre = 0;
    if (lane < kNS)
    {
#pragma unroll
        for (int w = 0; w < 4; ++w)
        {
            const int c = (int)pc.c[w][lane];
            t += c;
            pre += (w < wave) ? c : 0;
        }
    }
    int incl = t;
#pragma unroll
    for (int d = 1; d < 32; d *= 2)
    {
        const int y = __shfl_up(incl, d, 64);
        if (lane >= d) incl += y;
    }
    beg = incl - t;
    tot = t;
    base = beg + pre;
}

// Grid mode, f32, matrix-core form with per-entry tap tables (the hot path
// for W <= 16). A 64 x 64 tile per work item, 16 x 16 sub-tiles, four
// waves of 16-row bands each holding four sub-tiles' re / im in MFMA
// accumulators: the tile's update is a sum of rank-1 outer products
// ku (x) (kv w V), applied four visibilities per v_mfma_f32_16x16x4_f32.
// The ES taps are evaluated ONCE per bucketed entry, in chunks of CHUNK =
// 128 entries: thread t < 128 evaluates entry t's NTAP u-taps, thread
// t + 128 its v-taps and stores the weighted visibility (checkerboard sign
// folded in) once per entry, each with its own axis's tap range, band mask
// and table position. The tables are zero-padded: entry e's taps sit at
// kLead + e * kStride in rows of NTAP + 15 slots whose tail (and the lead
// before entry 0) stays zero, so the 16 rows (columns) of a sub-tile read
// taps d0 + i, d0 in [-15, NTAP), with no range check. A visit is {u index
// of row 0, v index of column 0} (the entry's word plus a per-(band,
// column block) constant) and the entry number, written by ballot
// compaction into the wave's list of each column block; the matrix loop
// forms the B operand as v-tap x visibility (the visibility read is a
// broadcast). Barriers are LDS-only and the next chunk's records load
// after this chunk's staging (no s_waitcnt vmcnt before the visit loops).
// Entries per chunk (<= 128: u taps staged by threads 0-127, v taps by
// 128-255; 256: both axes per thread). Real v-tap rows + one visibility
// per entry (round 5; the rows held v-tap x visibility as float2 before)
// take 31 KB of LDS per workgroup at W <= 8: 5 workgroups per CU instead
// of 4 (tile kernel 0.461 -> 0.447 ms at config 2, 26.1 -> 25.3 ms at
// config 3, 4.42 -> 4.24 ms for 10 w-planes).
constexpr int kScatterChunk = 128;
// w-planes per 3-D tile-kernel pass: 2 (10 planes: 1076 -> 1165 Mvis/s);
// 3 measured 1134 (162 VGPRs, 3 waves per SIMD, and a lone tenth plane).
constexpr int kScatterPlanes = 2;
// PLANES = 2 (3-D): w-planes p.plane and plane2 in one pass: the entries'
// u / v taps, lists and operand reads are shared, each visit feeds both
// planes' accumulators (visibility x w-tap of each plane), and the tile
// is written to grid and grid2.
template<bool DO_W, int NTAP, int CHUNK = kScatterChunk, int PLANES = 1>
__global__ __launch_bounds__(256) void k_scatter_tab(EsParams<float> p,
        const float* __restrict__ recs, const uint32_t* __restrict__ bin_start,
        const uint32_t* __restrict__ item_start,
        const uint32_t* __restrict__ item_bin, float* __restrict__ grid,
        int flags, float* __restrict__ grid2 = nullptr, int plane2 = 0,
        float* __restrict__ grid3 = nullptr)
{
    static_assert(PLANES == 1 || (PLANES <= 3 && DO_W), "planes 2, 3: 3-D");
    // (PLANES = 3 compiles and passed the 3-D tests, but loses: see
    // kScatterPlanes.)
    constexpr int kX = PLANES > 1 ? PLANES - 1 : 1;   // extra planes
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    static_assert(CHUNK == 256 || (CHUNK <= 128 && CHUNK % 16 == 0),
            "one or two threads per entry");
    constexpr int kHalf = CHUNK == 256 ? 256 : 128;   // threads per axis
    constexpr int kVec = DO_W ? 2 : 1;
    constexpr int kStride = NTAP + 15;
    constexpr int kLead = 16;
    constexpr int kTab = kLead + CHUNK * kStride;
    // Visit words hold byte offsets (u | v << 16) and the visibility's byte
    // offset, so a visit's three LDS addresses cost one packed 16-bit add,
    // an and and a shift (round 6; with table indices they took an and, a
    // bit-field extract, two shift-adds and a shift: tile kernel 0.439 ->
    // 0.420 ms at config 2, 25.1 -> 24.2 ms at config 3).
    constexpr uint32_t kPosUnit = 4, kVisUnit = 8;
    static_assert((kTab + 128) * kPosUnit < 65536, "16-bit table offsets");
    static_assert(kLead % 4 == 0 && kStride % 4 == 0, "16-byte table rows");
    __shared__ __attribute__((aligned(16))) float s_ku[kTab];
    __shared__ __attribute__((aligned(16))) float s_kv[kTab];
    __shared__ float2 s_vis[CHUNK + 1];   // [CHUNK]: zero, for padding visits
    __shared__ float2 s_visx[kX][PLANES > 1 ? CHUNK + 1 : 1];
    __shared__ uint2 s_list[4][CHUNK + 4];
    // Per entry: byte 0 = row bands hit, byte 1 = column blocks hit (0 for
    // entries past the chunk); s_pos: table byte offset of the entry's row
    // 0 / column 0 of the tile, + 64 taps (lo: u, hi: v). With CHUNK = 128 the u
    // half and the v half of both are written by the entry's two threads.
    __shared__ uint32_t s_info[CHUNK];
    __shared__ uint32_t s_pos[CHUNK];

    const uint32_t item = blockIdx.x;
    if (item_bin[item] == kNoBin) return;
    const int b = (int)item_bin[item];
    const uint32_t piece = item - item_start[b];
    const uint32_t npieces = item_start[b + 1] - item_start[b];
    const uint32_t e0 = bin_start[b] + piece * kPiece;
    const uint32_t e1 = min(bin_start[b + 1], e0 + kPiece);
    // flags bit 0 (skip_empty): a tile without entries is not written, its
    // consumer reads the bin counts; bit 1 (accumulate): batched call, the
    // tile is added to the grid (a work item without entries returns).
    const bool accumulate = (flags & 2) != 0;
    if ((flags & 1) && e0 == e1 && npieces == 1) return;
    if (accumulate && e0 == e1) return;
    int r0, c0;
    tile_origin(p, b, r0, c0);
    if (r0 >= p.G || c0 >= p.G) return;
    const int half = p.G / 2;
    const int tu0 = r0 - half, tv0 = c0 - half;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int i = lane & 15, kq = lane >> 4;
    const int sub_r = wave * 16;
    const uint32_t li4 = (uint32_t)(4 * i) * 0x10001u;   // (4 i, 4 i) bytes
    const int et = t & (kHalf - 1);               // this thread's entry
    const bool stage_u = CHUNK == 256 || t < 128;
    const bool stage_v = CHUNK == 256 || t >= 128;
    f32x4 acc_re[4], acc_im[4];
    f32x4 acc_rex[kX][PLANES > 1 ? 4 : 1], acc_imx[kX][PLANES > 1 ? 4 : 1];
#pragma unroll
    for (int cblk = 0; cblk < 4; ++cblk)
    {
        acc_re[cblk] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        acc_im[cblk] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
        if constexpr (PLANES > 1)
#pragma unroll
            for (int x = 0; x < kX; ++x)
            {
                acc_rex[x][cblk] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
                acc_imx[x][cblk] = f32x4{0.0f, 0.0f, 0.0f, 0.0f};
            }
    }
    for (int k = t; k < kTab; k += 256)
    {
        s_ku[k] = 0.0f;
        s_kv[k] = 0.0f;
    }
    if (t == 0)
    {
        s_vis[CHUNK] = make_float2(0.0f, 0.0f);
        if constexpr (PLANES > 1)
            for (int x = 0; x < kX; ++x)
                s_visx[x][CHUNK] = make_float2(0.0f, 0.0f);
    }
    const float4* recs4 = (const float4*)recs;
    float4 r = make_float4(0.0f, 0.0f, 0.0f, 0.0f), rw = r;
    if (et < CHUNK && e0 + et < e1)
    {
        r = recs4[(size_t)(e0 + et) * kVec];
        if (DO_W) rw = recs4[(size_t)(e0 + et) * kVec + 1];
    }
    for (uint32_t cb = e0; cb < e1; cb += CHUNK)
    {
        const int n = (int)min((uint32_t)CHUNK, e1 - cb);
        // Tap range of this thread's axis (both with CHUNK = 256): same
        // formula as tap_range / footprint.
        const float hs = (float)p.support / 2.0f;
        const int gmin = -p.G / 2, gmax = (p.G - 1) / 2;
        const bool live = et < n;
        int u0 = 0, u1 = -1, v0 = 0, v1 = -1;
        uint32_t rm = 0, cm = 0, pu16 = 0, pv16 = 0;
        const int eb = kLead + et * kStride;
        bool on_plane = live;
        float vxr[kX], vxi[kX];           // w V on the extra planes
        {
#pragma clang fp contract(off)
            if (DO_W)
            {
                // rw.x: the plane coordinate (bucketed for all planes);
                // an entry off this w-plane gets no visits.
                float kw = 0.0f;
                on_plane = live && plane_tap(p, rw.x, kw);
                if constexpr (PLANES > 1)
#pragma unroll
                    for (int x = 0; x < kX; ++x)
                    {
                        float kw2 = 0.0f;
                        on_plane = (live && plane_tap_at(p, plane2 + x, rw.x,
                                kw2)) || on_plane;
                        vxr[x] = r.z * kw2;
                        vxi[x] = r.w * kw2;
                    }
                r.z *= kw;
                r.w *= kw;
            }
            u0 = max((int)ceilf(r.x - hs), gmin);
            if (stage_u)
            {
                u1 = min((int)floorf(r.x + hs), gmax);
                const int lo = max(u0 - tu0, 0) >> 4;
                const int hi = min(u1 - tu0, kTile - 1) >> 4;
                rm = on_plane ? (2u << hi) - (1u << lo) : 0u;
                pu16 = (uint32_t)(eb + 64 - (u0 - tu0)) * kPosUnit;
            }
            if (stage_v)
            {
                v0 = max((int)ceilf(r.y - hs), gmin);
                v1 = min((int)floorf(r.y + hs), gmax);
                const int lo = max(v0 - tv0, 0) >> 4;
                const int hi = min(v1 - tv0, kTile - 1) >> 4;
                cm = on_plane ? (2u << hi) - (1u << lo) : 0u;
                pv16 = (uint32_t)(eb + 64 - (v0 - tv0)) * kPosUnit;
            }
        }
        lds_barrier();   // B1: previous chunk's tables and lists consumed
        if (CHUNK == 256)
        {
            s_info[et] = rm | cm << 8;
            s_pos[et] = pu16 | pv16 << 16;
        }
        else if (et < CHUNK)
        {
            uint8_t* info8 = (uint8_t*)s_info;
            uint16_t* pos16 = (uint16_t*)s_pos;
            info8[4 * et + (stage_u ? 0 : 1)] = (uint8_t)(stage_u ? rm : cm);
            pos16[2 * et + (stage_u ? 0 : 1)] = (uint16_t)(stage_u ? pu16 : pv16);
        }
        if (on_plane)
        {
#pragma clang fp contract(off)
            if (stage_u)
            {
                float tu[NTAP];
                axis_taps<NTAP, true>(p, r.x, u0, u1, tu);
                // 16-byte stores (eb is a multiple of 4): entry rows are
                // kStride = 24 words apart, so a wave's one-word stores of
                // tap d hit 8 banks (8-way conflicts); quads hit them 2-way.
                float4* q = reinterpret_cast<float4*>(s_ku + eb);
#pragma unroll
                for (int d = 0; d + 4 <= NTAP; d += 4)
                    q[d / 4] = make_float4(tu[d], tu[d + 1], tu[d + 2],
                            tu[d + 3]);
#pragma unroll
                for (int d = NTAP & ~3; d < NTAP; ++d) s_ku[eb + d] = tu[d];
            }
            if (stage_v)
            {
                float tv[NTAP];
                axis_taps<NTAP, true>(p, r.y, v0, v1, tv);
                const bool neg = ((u0 + v0) & 1) != 0;
                s_vis[et] = make_float2(neg ? -r.z : r.z, neg ? -r.w : r.w);
                if constexpr (PLANES > 1)
#pragma unroll
                    for (int x = 0; x < kX; ++x)
                        s_visx[x][et] = make_float2(neg ? -vxr[x] : vxr[x],
                                neg ? -vxi[x] : vxi[x]);
                float4* q = reinterpret_cast<float4*>(s_kv + eb);
#pragma unroll
                for (int d = 0; d + 4 <= NTAP; d += 4)
                    q[d / 4] = make_float4(tv[d], tv[d + 1], tv[d + 2],
                            tv[d + 3]);
#pragma unroll
                for (int d = NTAP & ~3; d < NTAP; ++d) s_kv[eb + d] = tv[d];
            }
        }
        // Next chunk's records, issued after this chunk's last use of r so
        // that nothing waits for them before the next staging.
        if (et < CHUNK && cb + CHUNK + et < e1)
        {
            r = recs4[(size_t)(cb + CHUNK + et) * kVec];
            if (DO_W) rw = recs4[(size_t)(cb + CHUNK + et) * kVec + 1];
        }
        lds_barrier();   // B2: entry words and tap tables complete

        uint2* list = s_list[wave];
        // A visit's operands: tap rows at byte offsets w.x + (4 i, 4 i)
        // (one packed 16-bit add; the halves do not carry into each other),
        // the weighted visibility at byte offset w.y.
        auto vis_at = [&](const float2* base, uint32_t off) -> float2 {
            return *reinterpret_cast<const float2*>(
                    reinterpret_cast<const char*>(base) + off);
        };
        auto visit_operands = [&](uint2 w, float& a, float& kv, float2& z) {
            typedef unsigned short us2 __attribute__((ext_vector_type(2)));
            const us2 ab = __builtin_bit_cast(us2, w.x) +
                    __builtin_bit_cast(us2, li4);
            const uint32_t abw = __builtin_bit_cast(uint32_t, ab);
            a = *reinterpret_cast<const float*>(
                    reinterpret_cast<const char*>(s_ku) + (abw & 0xffffu));
            kv = *reinterpret_cast<const float*>(
                    reinterpret_cast<const char*>(s_kv) + (abw >> 16));
            z = vis_at(s_vis, w.y);
        };
        // The chunk's entry words, read once for the four column blocks.
        constexpr int kGroups = (CHUNK + 63) / 64;
        // cbm: the column blocks an entry hits in this wave's row band.
        uint32_t cbm[kGroups], ps[kGroups];
#pragma unroll
        for (int gi = 0; gi < kGroups; ++gi)
        {
            const bool in = CHUNK % 64 == 0 || gi * 64 + lane < CHUNK;
            const uint32_t inf = in ? s_info[gi * 64 + lane] : 0u;
            cbm[gi] = ((inf >> wave) & 1u) ? (inf >> 8) & 0xFu : 0u;
            ps[gi] = in ? s_pos[gi * 64 + lane] : 0u;
        }
#pragma unroll
        for (int cblk = 0; cblk < 4; ++cblk)
        {
            // This wave's visits of sub-tile (wave, cblk), in entry order.
            // Visit word = entry word + 4 (sub_r - 64, cblk * 16 - 64)
            // bytes: both halves stay non-negative for a visited sub-tile,
            // so the one 32-bit add does not carry between them.
            const uint32_t kadd = (uint32_t)((sub_r - 64) * (int)kPosUnit) +
                    ((uint32_t)((cblk * 16 - 64) * (int)kPosUnit) << 16);
            int cnt = 0;
#pragma unroll
            for (int gi = 0; gi < kGroups; ++gi)
            {
                const bool hit = (cbm[gi] & (1u << cblk)) != 0u;
                const uint64_t m = __ballot(hit);
                // Slot cnt + (hits in lanes below): one mbcnt pair.
                if (hit)
                    list[__builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32),
                            __builtin_amdgcn_mbcnt_lo((uint32_t)m,
                            (uint32_t)cnt))] = make_uint2(ps[gi] + kadd,
                            (uint32_t)(gi * 64 + lane) * kVisUnit);
                cnt += (int)__popcll(m);
            }
            const int cnt4 = (cnt + 3) & ~3;
            if (lane < cnt4 - cnt)     // zero visit (zero taps, zero value)
                list[cnt + lane] = make_uint2(0u, (uint32_t)CHUNK * kVisUnit);
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
            const int n4 = __builtin_amdgcn_readfirstlane(cnt4);
            const int n16 = n4 & ~15;
            f32x4 re = acc_re[cblk], im = acc_im[cblk];
            f32x4 rex[kX], imx[kX];
            if constexpr (PLANES > 1)
#pragma unroll
                for (int x = 0; x < kX; ++x)
                {
                    rex[x] = acc_rex[x][cblk];
                    imx[x] = acc_imx[x][cblk];
                }
            for (int g = n16; g < n4; g += 4)
            {
                const uint2 w = list[g + kq];
                float a, kv;
                float2 z;
                visit_operands(w, a, kv, z);
                const float2 bb = make_float2(kv * z.x, kv * z.y);
                re = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb.x, re, 0, 0, 0);
                im = __builtin_amdgcn_mfma_f32_16x16x4f32(a, bb.y, im, 0, 0, 0);
                if constexpr (PLANES > 1)
#pragma unroll
                    for (int x = 0; x < kX; ++x)
                    {
                        const float2 z2 = vis_at(s_visx[x], w.y);
                        rex[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a,
                                kv * z2.x, rex[x], 0, 0, 0);
                        imx[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(a,
                                kv * z2.y, imx[x], 0, 0, 0);
                    }
            }
            for (int g = 0; g < n16; g += 16)
            {
                uint2 w[4];
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2) w[s2] = list[g + 4 * s2 + kq];
                float a[4];
                float2 bb[4];
                float2 bbx[kX][PLANES > 1 ? 4 : 1];
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2)
                {
                    float kv;
                    float2 z;
                    visit_operands(w[s2], a[s2], kv, z);
                    {
                        using f2v = __attribute__((ext_vector_type(2))) float;
                        const f2v pb = f2v{kv, kv} * f2v{z.x, z.y};
                        bb[s2] = make_float2(pb.x, pb.y);
                    }
                    if constexpr (PLANES > 1)
#pragma unroll
                        for (int x = 0; x < kX; ++x)
                        {
                            const float2 z2 = vis_at(s_visx[x], w[s2].y);
                            bbx[x][s2] = make_float2(kv * z2.x, kv * z2.y);
                        }
                }
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2)
                    re = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], bb[s2].x,
                            re, 0, 0, 0);
#pragma unroll
                for (int s2 = 0; s2 < 4; ++s2)
                    im = __builtin_amdgcn_mfma_f32_16x16x4f32(a[s2], bb[s2].y,
                            im, 0, 0, 0);
                if constexpr (PLANES > 1)
#pragma unroll
                    for (int x = 0; x < kX; ++x)
                    {
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2)
                            rex[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                    a[s2], bbx[x][s2].x, rex[x], 0, 0, 0);
#pragma unroll
                        for (int s2 = 0; s2 < 4; ++s2)
                            imx[x] = __builtin_amdgcn_mfma_f32_16x16x4f32(
                                    a[s2], bbx[x][s2].y, imx[x], 0, 0, 0);
                    }
            }
            acc_re[cblk] = re;
            acc_im[cblk] = im;
            if constexpr (PLANES > 1)
#pragma unroll
                for (int x = 0; x < kX; ++x)
                {
                    acc_rex[x][cblk] = rex[x];
                    acc_imx[x][cblk] = imx[x];
                }
            // The list is rebuilt for the next column block.
            __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront", "local");
            __builtin_amdgcn_wave_barrier();
            __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront", "local");
        }
    }
    auto write_tile = [&](float* __restrict__ g, const f32x4 (&ar)[4],
            const f32x4 (&ai)[4]) {
        // A tile owned whole by this work item and inside the grid (every
        // tile when G is a multiple of 64): straight-line stores, no
        // per-element bounds or mode branches.
        if (npieces == 1 && r0 + 64 <= p.G && c0 + 64 <= p.G)
        {
            float* base = g + ((size_t)(r0 + sub_r + kq * 4) * p.G + c0 + i) * 2;
            if (accumulate)
            {
#pragma unroll
                for (int cblk = 0; cblk < 4; ++cblk)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                    {
                        float* dst = base + ((size_t)rr * p.G + cblk * 16) * 2;
                        float2 v = *(const float2*)dst;
                        v.x += ar[cblk][rr];
                        v.y += ai[cblk][rr];
                        *(float2*)dst = v;
                    }
            }
            else
            {
#pragma unroll
                for (int cblk = 0; cblk < 4; ++cblk)
#pragma unroll
                    for (int rr = 0; rr < 4; ++rr)
                    {
                        float* dst = base + ((size_t)rr * p.G + cblk * 16) * 2;
                        *(float2*)dst = make_float2(ar[cblk][rr], ai[cblk][rr]);
                    }
            }
            return;
        }
#pragma unroll
        for (int cblk = 0; cblk < 4; ++cblk)
        {
            const int col = c0 + cblk * 16 + i;
#pragma unroll
            for (int rr = 0; rr < 4; ++rr)
            {
                const int row = r0 + sub_r + kq * 4 + rr;
                if (row >= p.G || col >= p.G) continue;
                float* dst = g + ((size_t)row * p.G + col) * 2;
                if (npieces == 1 && accumulate)
                {
                    float2 v = *(const float2*)dst;
                    v.x += ar[cblk][rr];
                    v.y += ai[cblk][rr];
                    *(float2*)dst = v;
                }
                else if (npieces == 1)
                {
                    float2 v;
                    v.x = ar[cblk][rr];
                    v.y = ai[cblk][rr];
                    *(float2*)dst = v;
                }
                else
                {
                    if (ar[cblk][rr] != 0.0f)
                        unsafeAtomicAdd(dst, ar[cblk][rr]);
                    if (ai[cblk][rr] != 0.0f)
                        unsafeAtomicAdd(dst + 1, ai[cblk][rr]);
                }
            }
        }
    };
    write_tile(grid, acc_re, acc_im);
    if constexpr (PLANES > 1) write_tile(grid2, acc_rex[0], acc_imx[0]);
    if constexpr (PLANES > 2) write_tile(grid3, acc_rex[1], acc_imx[1]);
}

// Degrid mode, f32, matrix-core form with per-entry tap tables (the hot
// path for W <= 16).
//
// For visibility j and a 16x16 sub-tile (rows R, cols C) of the grid,
//   partial_j = sum_r s_u ku_j[r] * (sum_c G[r][c] s_v kv_j[c])
// The inner sums for 16 visibilities at once are T = G_sub * Kv, a
// 16x16x16 product = four v_mfma_f32_16x16x4_f32 per re / im, with the
// sub-tile's grid values as the A operand (loaded once per sub-tile from
// the LDS window) and B[c][j] = the v-taps of visibility j. In the C
// layout lane l holds T[4(l>>4)+r][l&15], so it applies four u-taps of
// visibility l&15, and a two-step lane-group reduction gives partial_j.
// Entries are bucketed by the tile of their first tap, so a tile's
// entries reach into the next 16 rows / cols: the workgroup stages the
// 80x80 window (tile + halo) in LDS and works on 5x5 sub-tiles; partials
// of one visibility from several sub-tiles meet in an LDS accumulator
// (16-lane ds_add_f32), and each visibility is read-modify-written in HBM
// once.
// Each entry's NTAP u-taps and v-taps (checkerboard sign folded in) are
// evaluated once at staging into LDS tables; visits are packed {entry,
// u0 - tile row, v0 - tile col} words; the pool is laid out without atomics
// and the next chunk's records are prefetched.
template<bool DO_W, int NTAP>
__global__ __launch_bounds__(256) void k_gather_tab(EsParams<float> p,
        const float* __restrict__ recs, const uint32_t* __restrict__ bin_start,
        const uint32_t* __restrict__ item_start,
        const uint32_t* __restrict__ item_bin, const float* __restrict__ grid,
        float* __restrict__ vis)
{
    using f32x4 = __attribute__((ext_vector_type(4))) float;
    constexpr int kChunk = 256;
    constexpr int kSub = 5;                 // 5 x 5 sub-tiles: tile + halo
    constexpr int kZero = kChunk * NTAP;    // zero element for masked lanes
    __shared__ uint32_t s_pool[4 * kChunk]; // packed visits
    __shared__ float s_ku[kChunk * NTAP + 1];
    __shared__ float s_kv[kChunk * NTAP + 1];
    __shared__ float s_kw[kChunk];
    __shared__ float s_acc_re[kChunk];
    __shared__ float s_acc_im[kChunk];
    __shared__ PoolCounts<kSub * kSub> s_pc;

    const uint32_t item = blockIdx.x;
    if (item_bin[item] == kNoBin) return;   // past the last work item
    const int b = (int)item_bin[item];
    const uint32_t piece = item - item_start[b];
    const uint32_t e0 = bin_start[b] + piece * kPiece;
    const uint32_t e1 = min(bin_start[b + 1], e0 + kPiece);
    if (e0 >= e1) return;   // empty tile
    const int half = p.G / 2;
    int r0, c0;
    tile_origin(p, b, r0, c0);
    if (r0 >= p.G || c0 >= p.G) return;    // phantom tile
    const int tu0 = r0 - half, tv0 = c0 - half;
    const float2* g2 = (const float2*)grid;
    const int t = threadIdx.x;
    const int lane = t & 63, wave = t >> 6;
    const int jl = lane & 15, kq = lane >> 4;
    const float4* recs4 = (const float4*)recs;
    if (t == 0)
    {
        s_ku[kZero] = 0.0f;
        s_kv[kZero] = 0.0f;
    }
    float4 r = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (e0 + t < e1) r = recs4[e0 + t];

    for (uint32_t cb = e0; cb < e1; cb += kChunk)
    {
        const int n = (int)min((uint32_t)kChunk, e1 - cb);
        float4 rn = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (cb + kChunk + t < e1) rn = recs4[cb + kChunk + t];   // prefetch
        int wlo_r = 1, whi_r = 0, wlo_c = 1, whi_c = 0;
        int u0 = 0, u1 = -1, v0 = 0, v1 = -1;
        uint32_t pk = 0;
        // 3-D: records carry the plane coordinate (|r.z|); an entry off
        // this w-plane gets no visits and no write-back.
        float kw = 1.0f;
        const bool on_plane = t < n &&
                (!DO_W || plane_tap(p, fabsf(r.z), kw));
        if (on_plane)
        {
            tap_range(p, r.x, r.y, u0, u1, v0, v1);
            wlo_r = (u0 - tu0) >> 4;
            whi_r = min(u1 - tu0, kSub * 16 - 1) >> 4;
            wlo_c = (v0 - tv0) >> 4;
            whi_c = min(v1 - tv0, kSub * 16 - 1) >> 4;
            pk = (uint32_t)t | (uint32_t)(u0 - tu0) << 8 |
                    (uint32_t)(v0 - tv0) << 16;
        }
        int sub[4], rank[4];
        pool_count<kSub>(s_pc, lane, wave, wlo_r, whi_r, wlo_c, whi_c, sub,
                rank);
        __syncthreads();   // B1: previous chunk consumed
        if (on_plane)
        {
#pragma clang fp contract(off)
            float tu[NTAP], tv[NTAP];
            axis_taps<NTAP, false>(p, r.x, u0, u1, tu);
            axis_taps<NTAP, false>(p, r.y, v0, v1, tv);
#pragma unroll
            for (int d = 0; d < NTAP; ++d)
            {
                s_ku[t * NTAP + d] = tu[d];
                s_kv[t * NTAP + d] = tv[d];
            }
            // (-1)^(u0 + v0) of the checkerboard, with the w-tap
            s_kw[t] = ((u0 + v0) & 1) ? -kw : kw;
        }
        s_acc_re[t] = 0.0f;
        s_acc_im[t] = 0.0f;
        __syncthreads();   // B2: counts, tables, accumulators ready
        int beg_l, tot_l, base_l;
        pool_layout<kSub * kSub>(s_pc, lane, wave, beg_l, tot_l, base_l);
#pragma unroll
        for (int k = 0; k < 4; ++k)
        {
            const int pos = __shfl(base_l, max(sub[k], 0), 64) + rank[k];
            if (sub[k] >= 0) s_pool[pos] = pk;
        }
        __syncthreads();   // B3: pool complete
        for (int st = wave; st < kSub * kSub; st += 4)
        {
            const int sts = __builtin_amdgcn_readfirstlane(st);
            const int cnt = __builtin_amdgcn_readlane(tot_l, sts);
            if (cnt == 0) continue;
            const int v_beg = __builtin_amdgcn_readlane(beg_l, sts);
            const int R0 = (sts / kSub) * 16, C0 = (sts % kSub) * 16;
            // A operands straight from the grid (L2 / HBM):
            // G[r0 + R0 + jl][c0 + C0 + 4 kk + kq], kk = 0..3.
            float a_re[4], a_im[4];
            const int grow = r0 + R0 + jl;
#pragma unroll
            for (int kk = 0; kk < 4; ++kk)
            {
                const int gcol = c0 + C0 + 4 * kk + kq;
                float2 v = make_float2(0.0f, 0.0f);
                if (grow < p.G && gcol < p.G) v = g2[(size_t)grow * p.G + gcol];
                a_re[kk] = v.x;
                a_im[kk] = v.y;
            }
            for (int g = 0; g < cnt; g += 16)
            {
#pragma clang fp contract(off)
                const bool valid = g + jl < cnt;
                const uint32_t q = s_pool[v_beg + (valid ? g + jl : cnt - 1)];
                const int e = (int)(q & 0xffu);
                const int eb = e * NTAP;
                const int ou = (int)((q >> 8) & 0xffu), ov = (int)(q >> 16);
                f32x4 t_re = {0.0f, 0.0f, 0.0f, 0.0f};
                f32x4 t_im = {0.0f, 0.0f, 0.0f, 0.0f};
                float kv[4], ku[4];
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                {
                    const int dv = C0 + 4 * kk + kq - ov;
                    kv[kk] = s_kv[((unsigned)dv < (unsigned)NTAP) ? eb + dv :
                            kZero];
                    const int du = R0 + 4 * kq + kk - ou;
                    ku[kk] = s_ku[(valid && (unsigned)du < (unsigned)NTAP) ?
                            eb + du : kZero];
                }
#pragma unroll
                for (int kk = 0; kk < 4; ++kk)
                {
                    t_re = __builtin_amdgcn_mfma_f32_16x16x4f32(a_re[kk],
                            kv[kk], t_re, 0, 0, 0);
                    t_im = __builtin_amdgcn_mfma_f32_16x16x4f32(a_im[kk],
                            kv[kk], t_im, 0, 0, 0);
                }
                float p_re = 0.0f, p_im = 0.0f;
#pragma unroll
                for (int rr = 0; rr < 4; ++rr)
                {
                    p_re += ku[rr] * t_re[rr];
                    p_im += ku[rr] * t_im[rr];
                }
                // Sum the four lane groups (rows 4kq..4kq+3).
                p_re = sdp_hip::sum_rows16(p_re);
                p_im = sdp_hip::sum_rows16(p_im);
                if (kq == 0 && valid)
                {
                    const float kw = s_kw[e];
                    atomicAdd(&s_acc_re[e], p_re * kw);
                    atomicAdd(&s_acc_im[e], p_im * kw);
                }
            }
        }
        __syncthreads();
        if (on_plane)
        {
            const uint64_t idx = (uint64_t)__float_as_uint(r.w);
            const float flip = signbit(r.z) ? -1.0f : 1.0f;
            vis[2 * idx] += s_acc_re[t];
            vis[2 * idx + 1] += s_acc_im[t] * flip;   // kernels.cu:267-268
        }
        r = rn;
    }
}

// Degrid mode, f32, lane-per-entry form (the default for W <= 8). A work
// item stages the grid window its entries can reach -- the 64 x 64 tile of
// their first taps plus the 8 cells a 9-tap support extends past it --
// into LDS with coalesced row loads, then each thread gathers whole
// entries: the entry's u and v taps are evaluated once (polynomial
// interior taps, as the scatter), the 8 (or 9) grid rows of its support
// are contracted with the v taps and the row sums with the u taps, and the
// visibility is read-modify-written once. Work per entry: 64 LDS reads and
// 144 FMAs, with no cross-lane reduction, no sub-tile pools and no record
// sort; the matrix-core form (k_gather_tab) spends 16 x 16 products per
// sub-tile visit on 8 x 8 supports.
// ROWS: the tile rows one workgroup serves (64, or 32: each work item is
// split over two workgroups by the row of the entries' first tap, so the
// window is 40 x 72 and twice as many workgroups share a CU); NT threads.
template<bool DO_W, int NTAP, int ROWS, int NT>
__global__ __launch_bounds__(NT) void k_gather_win(EsParams<float> p,
        const float* __restrict__ recs, const uint32_t* __restrict__ bin_start,
        const uint32_t* __restrict__ item_start,
        const uint32_t* __restrict__ item_bin, const float* __restrict__ grid,
        float* __restrict__ vis)
{
    static_assert(NTAP == 9, "window of tile + 8 cells");
    static_assert(kTile % ROWS == 0, "whole parts of a tile");
    constexpr int kParts = kTile / ROWS;
    constexpr int kWin = kTile + NTAP - 1;     // 72 columns
    constexpr int kWinR = ROWS + NTAP - 1;     // window rows
    constexpr int kPitch = kWin;               // float2 per LDS row
    __shared__ float2 win[kWinR * kPitch];
    const uint32_t item = blockIdx.x / kParts;
    const int part = (int)(blockIdx.x % kParts);
    if (item_bin[item] == kNoBin) return;      // past the last work item
    const int b = (int)item_bin[item];
    const uint32_t piece = item - item_start[b];
    const uint32_t e0 = bin_start[b] + piece * kPiece;
    const uint32_t e1 = min(bin_start[b + 1], e0 + kPiece);
    if (e0 >= e1) return;                      // empty tile
    int r0, c0;
    tile_origin(p, b, r0, c0);
    if (r0 >= p.G || c0 >= p.G) return;        // phantom tile
    const int t = threadIdx.x;
    const int half = p.G / 2;
    const int tu0 = r0 - half, tv0 = c0 - half;
    const int rw0 = r0 + part * ROWS;          // first window row (grid)
    const int ru_lo = part * ROWS;             // entries' first-tap rows
    // This thread's first record, in flight during the window staging.
    const float4* recs4 = (const float4*)recs;
    float4 r = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    if (e0 + t < e1) r = recs4[e0 + t];
    // The window as 16-byte loads (two cells; c0 and G are even), all of a
    // thread's loads issued before the first LDS store: one memory latency
    // per work item instead of one per loop trip. Buffer loads relative to
    // the window's first row (32-bit offsets for any G); cells past the grid
    // address beyond the range and load zeros.
    {
        constexpr int kQ = kWin / 2;                 // float4 per window row
        constexpr int kN4 = kWinR * kQ;
        constexpr int kPer = (kN4 + NT - 1) / NT;
        const size_t row_f2 = (size_t)p.G;
        const float* wbase = grid + 2 * (size_t)rw0 * row_f2;
        const uint32_t nrows = (uint32_t)min(kWinR, p.G - rw0);
        const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(
                const_cast<float*>(wbase), 0, (int)(nrows * row_f2 * 8u),
                0x00020000);
        float4 wv[kPer];
#pragma unroll
        for (int j = 0; j < kPer; ++j)
        {
            const int k = t + j * NT;
            const int rr = k / kQ, cq = k - rr * kQ;
            const bool in = k < kN4 && c0 + 2 * cq < p.G;
            const uint32_t off = in ? (uint32_t)((rr * row_f2 + c0 + 2 * cq)
                    * 8u) : 0xFFFFFFF0u;
            wv[j] = __builtin_bit_cast(float4,
                    __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 0));
        }
#pragma unroll
        for (int j = 0; j < kPer; ++j)
        {
            const int k = t + j * NT;
            const int rr = k / kQ, cq = k - rr * kQ;
            if (k < kN4)
                *reinterpret_cast<float4*>(&win[rr * kPitch + 2 * cq]) = wv[j];
        }
    }
    __syncthreads();
    for (uint32_t e = e0 + t; e < e1; e += NT)
    {
#pragma clang fp contract(off)
        const float4 rc = r;
        if (e + NT < e1) r = recs4[e + NT];
        float kw = 1.0f;
        if (DO_W && !plane_tap(p, fabsf(rc.z), kw)) continue;   // off plane
        int u0, u1, v0, v1;
        tap_range(p, rc.x, rc.y, u0, u1, v0, v1);
        if (kParts > 1 && (unsigned)(u0 - tu0 - ru_lo) >= (unsigned)ROWS)
            continue;                          // the other part's entry
        // The visibility's current value, loaded before the taps and the
        // contraction so that its latency overlaps them (the entry is the
        // visibility's only one: degrid records sit in the tile of their
        // first tap). Read at the end, its round trip and the store's
        // completion sat in every iteration.
        const uint64_t idx = (uint64_t)__float_as_uint(rc.w);
        float2* vdst = reinterpret_cast<float2*>(vis + 2 * idx);
        const float2 vold = *vdst;
        float tu[NTAP], tv[NTAP];
        axis_taps<NTAP, true>(p, rc.x, u0, u1, tu);
        axis_taps<NTAP, true>(p, rc.y, v0, v1, tv);
        const float2* base = win + (u0 - tu0 - ru_lo) * kPitch + (v0 - tv0);
        float sr = 0.0f, si = 0.0f;
        // 2-D: the unrolled form (92 VGPRs, 5 waves per SIMD) measured
        // 447 -> 438 us at config 2; 3-D (plane-tap divergence): the row
        // loop (70 VGPRs, 7 waves) 391 vs 403 us.
        if constexpr (!DO_W)
        {
            // The ninth tap of an axis is non-zero only at an exact-integer
            // position (W + 1 taps, rare): the wave takes the 9 x 9 form
            // only if one of its entries has one (taps past u1 / v1 are zero
            // and the window holds the rows / columns they address), else
            // 8 x 8. Fully unrolled: tap registers with constant indices.
            const bool nine = u1 - u0 + 1 == NTAP || v1 - v0 + 1 == NTAP;
            auto contract = [&](auto n_c) {
                constexpr int N = decltype(n_c)::value;
#pragma unroll
                for (int du = 0; du < N; ++du)
                {
                    const float2* row = base + du * kPitch;
                    float tr = 0.0f, ti = 0.0f;
#pragma unroll
                    for (int dv = 0; dv < N; ++dv)
                    {
                        const float2 g = row[dv];
                        tr = __builtin_fmaf(tv[dv], g.x, tr);
                        ti = __builtin_fmaf(tv[dv], g.y, ti);
                    }
                    sr = __builtin_fmaf(tu[du], tr, sr);
                    si = __builtin_fmaf(tu[du], ti, si);
                }
            };
            if (__ballot(nine))
                contract(std::integral_constant<int, NTAP>{});
            else
                contract(std::integral_constant<int, NTAP - 1>{});
        }
        else
        {
            // The ninth tap of an axis is non-zero only at an exact-integer
            // position (W + 1 taps); rows / columns of zero taps are skipped.
            const int nu = u1 - u0 + 1, nv = v1 - v0 + 1;
#pragma unroll
            for (int du = 0; du < NTAP; ++du)
            {
                if (du >= nu) break;
                const float2* row = base + du * kPitch;
                float tr = 0.0f, ti = 0.0f;
#pragma unroll
                for (int dv = 0; dv < NTAP - 1; ++dv)
                {
                    const float2 g = row[dv];
                    tr = __builtin_fmaf(tv[dv], g.x, tr);
                    ti = __builtin_fmaf(tv[dv], g.y, ti);
                }
                if (nv == NTAP)
                {
                    const float2 g = row[NTAP - 1];
                    tr = __builtin_fmaf(tv[NTAP - 1], g.x, tr);
                    ti = __builtin_fmaf(tv[NTAP - 1], g.y, ti);
                }
                sr = __builtin_fmaf(tu[du], tr, sr);
                si = __builtin_fmaf(tu[du], ti, si);
            }
        }
        // (-1)^(u0 + v0) of the checkerboard, with the w-tap; the flip
        // conjugates (kernels.cu:267-268).
        const float ks = ((u0 + v0) & 1) ? -kw : kw;
        const float flip = signbit(rc.z) ? -1.0f : 1.0f;
        *vdst = make_float2(vold.x + sr * ks, vold.y + si * ks * flip);
    }
}

// Degrid mode: one workgroup per work item; the tile plus its support halo
// is staged in LDS once. Records are loaded 64 per wave; taps of four
// entries are evaluated cooperatively; each entry is gathered by the whole
// wave (lane = tap) and reduced with a butterfly; lane j keeps entry j's sum
// so the batch's visibilities are updated by one scattered RMW per lane.
template<typename T, bool DO_W>
__global__ __launch_bounds__(kThreads) void k_gather(EsParams<T> p,
        const T* __restrict__ recs, const uint32_t* __restrict__ bin_start,
        const uint32_t* __restrict__ item_start,
        const uint32_t* __restrict__ item_bin, const T* __restrict__ grid,
        T* __restrict__ vis, int wrows, int ws)
{
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    T* w_re = (T*)smem;
    T* w_im = w_re + wrows * ws;
    const uint32_t item = blockIdx.x;
    if (item_bin[item] == kNoBin) return;   // past the last work item
    const int b = (int)item_bin[item];
    const uint32_t piece = item - item_start[b];
    const uint32_t e0 = bin_start[b] + piece * kPiece;
    const uint32_t e1 = min(bin_start[b + 1], e0 + kPiece);
    if (e0 >= e1) return;   // empty tile: nothing to gather
    const int half = p.G / 2;
    int r0, c0;
    tile_origin(p, b, r0, c0);
    if (r0 >= p.G || c0 >= p.G) return;    // phantom tile
    const int tu0 = r0 - half, tv0 = c0 - half;
    using T2 = typename Vec2<T>::type;
    const T2* g2 = (const T2*)grid;
    for (int k = threadIdx.x; k < wrows * wrows; k += kThreads)
    {
        const int r = k / wrows, c = k - r * wrows;
        T2 val;
        val.x = T(0);
        val.y = T(0);
        if (r0 + r < p.G && c0 + c < p.G)
            val = g2[(size_t)(r0 + r) * p.G + c0 + c];
        w_re[r * ws + c] = val.x;
        w_im[r * ws + c] = val.y;
    }
    __syncthreads();

    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int du = lane >> 3, dv = lane & 7;
    const int lane_off = du * ws + dv;
    const int lane_par = (du + dv) & 1;
    const T inv_hs = T(1) / (T(p.support) / T(2));
    for (uint32_t base = e0 + wave * 64; base < e1; base += kWaves * 64)
    {
        Batch<T> bt;
        // Gather records are {pu, pv, kw*flip, index}: kw = |a|.
        load_batch<T, false, 4>(p, recs, base, e1, lane, tu0, tv0, wrows, bt);
        // 3-D: |a| is the plane coordinate (bucketed for all planes).
        const T pw = fabs(bt.a);
        T kw_lane = pw;
        if (DO_W) (void)plane_tap(p, pw, kw_lane);   // 0 off this plane
        T res_re = T(0), res_im = T(0);
        for (int g = 0; g < bt.cnt; g += 4)
        {
            const T es = group_taps(p, bt, g, lane, inv_hs);
#pragma unroll
            for (int jj = 0; jj < 4; ++jj)
            {
                const int j = g + jj;
                if (j >= bt.cnt) break;
                const T ku = __shfl(es, (jj << 4) | du);
                const T kv = __shfl(es, (jj << 4) | 8 | dv);
                const T kw = DO_W ? lane_bcast(kw_lane, j) : T(1);
                T acc_re = T(0), acc_im = T(0);
                if ((bt.wide >> j) & 1ull)
                {
                    const T pu = lane_bcast(bt.pu, j), pv = lane_bcast(bt.pv, j);
                    int u0, u1, v0, v1;
                    tap_range(p, pu, pv, u0, u1, v0, v1);
                    for (int ub = u0; ub <= u1; ub += 8)
                        for (int vb = v0; vb <= v1; vb += 8)
                        {
                            const int u = ub + du, v = vb + dv;
                            if (u <= u1 && v <= v1)
                            {
                                const T k = tap_weight(p, u, v, pu, pv, kw);
                                const int a = (u - tu0) * ws + (v - tv0);
                                acc_re += w_re[a] * k;
                                acc_im += w_im[a] * k;
                            }
                        }
                }
                else
                {
                    const int win = lane_bcast(bt.win, j);
                    const int org = lane_bcast(bt.org, j);
                    const bool act = du >= (win & 255) &&
                            du < ((win >> 8) & 255) &&
                            dv >= ((win >> 16) & 255) && dv < (win >> 24);
                    T k = ku * kv;
                    if (DO_W) k *= kw;
                    if ((lane_par + org + (org >> 16)) & 1) k = -k;
                    if (act)
                    {
                        const int a = lane_off + ((org & 0xffff) - 256) * ws +
                                ((org >> 16) - 256);
                        acc_re = w_re[a] * k;
                        acc_im = w_im[a] * k;
                    }
                }
#pragma unroll
                for (int off = 32; off > 0; off >>= 1)
                {
                    acc_re += __shfl_xor(acc_re, off);
                    acc_im += __shfl_xor(acc_im, off);
                }
                if (lane == j)
                {
                    res_re = acc_re;
                    res_im = acc_im;
                }
            }
        }
        if (lane < bt.cnt)
        {
            const uint64_t i = bits_idx(bt.b);
            const T flip = signbit(bt.a) ? T(-1) : T(1);
            vis[2 * i] += res_re;
            vis[2 * i + 1] += res_im * flip;   // kernels.cu:267-268
        }
    }
}

// Image-plane kernels ---------------------------------------------------------


template<typename T>
__global__ void k_screen_corr_2d(ImageParams<T> ip, const T* __restrict__ layer,
        T* __restrict__ dirty)
{
#pragma clang fp contract(off)
    const int h = ip.N / 2;
    const int ix = blockIdx.x * blockDim.x + threadIdx.x;
    const int iy = blockIdx.y * blockDim.y + threadIdx.y;
    if (ix >= 2 * h || iy >= 2 * h) return;
    const int x = ix - h, y = iy - h, gc = ip.G / 2;
    T val = layer[((size_t)(gc + y) * ip.G + (gc + x)) * 2];
    if ((ix + iy) & 1) val = -val;
    T* d = dirty + (size_t)iy * ip.N + ix;
    T out = *d + val;
    out *= inv_correction(ip, abs(x), abs(y));
    *d = out;
}

template<typename T>
__global__ void k_screen_accumulate(ImageParams<T> ip, int plane,
        const T* __restrict__ layer, T* __restrict__ dirty)
{
#pragma clang fp contract(off)
    const int h = ip.N / 2;
    const int ix = blockIdx.x * blockDim.x + threadIdx.x;
    const int iy = blockIdx.y * blockDim.y + threadIdx.y;
    if (ix >= 2 * h || iy >= 2 * h) return;
    const int x = ix - h, y = iy - h, gc = ip.G / 2;
    const size_t g = ((size_t)(gc + y) * ip.G + (gc + x)) * 2;
    T re, im;
    phasor(ip, plane, abs(x), abs(y), T(-1), re, im);
    T val = layer[g] * re - layer[g + 1] * im;
    if ((ix + iy) & 1) val = -val;
    dirty[(size_t)iy * ip.N + ix] += val;
}

template<typename T>
__global__ void k_apply_correction(ImageParams<T> ip, T* __restrict__ dirty)
{
    // The correction depends on |x - h|, |y - h| only: one evaluation per
    // offset pair (i, j), applied to the up to four pixels h +- i, h +- j
    // of the image (rows and columns < 2h).
    const int h = ip.N / 2;
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    const int j = blockIdx.y * blockDim.y + threadIdx.y;
    if (i > h || j > h) return;
    const T f = inv_correction(ip, i, j);
    const int xs[2] = {h - i, h + i}, ys[2] = {h - j, h + j};
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 2; ++b)
        {
            const int ix = xs[b], iy = ys[a];
            if ((a && j == 0) || (b && i == 0) || ix >= 2 * h || iy >= 2 * h)
                continue;
            dirty[(size_t)iy * ip.N + ix] *= f;
        }
}

// Whole-grid writer for degridding: centre = checker * dirty * phasor.
template<typename T>
__global__ void k_reverse_screen(ImageParams<T> ip, int plane,
        T* __restrict__ dirty, int correct_in_place, T* __restrict__ grid)
{
#pragma clang fp contract(off)
    const int gx = blockIdx.x * blockDim.x + threadIdx.x;
    const int gy = blockIdx.y * blockDim.y + threadIdx.y;
    if (gx >= ip.G || gy >= ip.G) return;
    const int h = ip.N / 2, gc = ip.G / 2;
    const int x = gx - gc, y = gy - gc;
    T re = T(0), im = T(0);
    if (x >= -h && x < h && y >= -h && y < h)
    {
        T* d = dirty + (size_t)(y + h) * ip.N + (x + h);
        T val = *d;
        if (correct_in_place)
        {
            val *= inv_correction(ip, abs(x), abs(y));
            *d = val;
        }
        if ((x + y) & 1) val = -val;
        T pr = T(1), pi = T(0);
        if (ip.do_w) phasor(ip, plane, abs(x), abs(y), T(1), pr, pi);
        re = pr * val;
        im = pi * val;
    }
    T* g = grid + ((size_t)gy * ip.G + gx) * 2;
    g[0] = re;
    g[1] = im;
}

// hipFuncSetAttribute is a host call with real latency: do it once per
// kernel instantiation, not per launch (it would otherwise leave the GPU
// idle between the bucketing and the tile kernel).
template<auto Kernel>
int allow_lds(size_t bytes)
{
    static int done_bytes = 0;   // one per kernel instantiation
    if ((int)bytes <= done_bytes) return hipSuccess;
    const hipError_t e = hipFuncSetAttribute((const void*)Kernel,
            hipFuncAttributeMaxDynamicSharedMemorySize, (int)bytes);
    if (e == hipSuccess) done_bytes = (int)bytes;
    return e;
}

dim3 image_blocks(int n)
{
    return dim3((unsigned)((n + 63) / 64), (unsigned)((n + 3) / 4));
}

} // namespace

void es_tap_poly_fit(double beta, float out[kTapPolyPairs]
        [kTapPolyDeg + 1][2])
{
    // Interior taps d = 1..6 of W = 8 (half support 4):
    //   psi_d(s) = exp(beta (sqrt(1 - x^2) - 1)), x = ((s + 1) / 2 + d) / 4 - 1
    // interpolated at the Chebyshev nodes of degree n - 1 in double, then
    // expanded into monomials of s, with (-1)^d folded in.
    constexpr int n = kTapPolyDeg + 1;
    const double pi = 3.14159265358979323846;
    for (int d = 1; d <= 2 * kTapPolyPairs; ++d)
    {
        double f[n], a[n];
        for (int k = 0; k < n; ++k)
        {
            const double sk = cos(pi * (k + 0.5) / n);
            const double x = ((sk + 1.0) / 2.0 + d) / 4.0 - 1.0;
            f[k] = exp(beta * (sqrt(1.0 - x * x) - 1.0));
        }
        for (int j = 0; j < n; ++j)
        {
            double acc = 0.0;
            for (int k = 0; k < n; ++k)
                acc += f[k] * cos(pi * j * (k + 0.5) / n);
            a[j] = acc * 2.0 / n;
        }
        a[0] *= 0.5;
        // sum_j a_j T_j(s) -> monomials, T_{j+1} = 2 s T_j - T_{j-1}.
        double mono[n] = {0.0}, tm1[n] = {0.0}, t0[n] = {0.0}, t1[n];
        t0[0] = 1.0;                       // T_0
        for (int j = 0; j < n; ++j)
        {
            for (int k = 0; k < n; ++k) mono[k] += a[j] * t0[k];
            for (int k = 0; k < n; ++k)
                t1[k] = (k > 0 ? (j == 0 ? 1.0 : 2.0) * t0[k - 1] : 0.0) -
                        (j == 0 ? 0.0 : tm1[k]);
            for (int k = 0; k < n; ++k)
            {
                tm1[k] = t0[k];
                t0[k] = t1[k];
            }
        }
        const double sign = (d & 1) ? -1.0 : 1.0;
        for (int k = 0; k < n; ++k)
            out[(d - 1) / 2][k][(d - 1) % 2] = (float)(sign * mono[k]);
    }
}

// Visibilities per bucketing chunk: 8192 beat 12 k / 16 k / 32 k (fewer
// blocks hurt both record levels).
constexpr int64_t kChunkVis = 8192;

int num_chunks(int64_t num_vis, int tstride)
{
    const int64_t cv = kChunkVis;
    const int64_t by_size = (num_vis + cv - 1) / cv;
    const int64_t by_table = (((int64_t)1 << 31) - 1) /
            (4 * (int64_t)std::max(1, tstride));
    return (int)std::max<int64_t>(1, std::min<int64_t>(
            std::min<int64_t>(kMaxChunks, by_table), by_size));
}

size_t bucket_table_entries(int nc, int nbins, int nsbins)
{
    const size_t ng = (size_t)(nc + kGroupChunks - 1) / kGroupChunks;
    return (size_t)nc * nsbins + ng * nbins;
}

bool super_geometry(int ntiles, int* sshift, int* nsuper, int* nsbins)
{
    for (int sh = 3; (1 << (2 * sh)) <= kMaxSuperTiles; ++sh)
    {
        const int n = (ntiles + (1 << sh) - 1) >> sh;
        if (n * n <= kMaxSuperBins)
        {
            *sshift = sh;
            *nsuper = n;
            *nsbins = n * n;
            return true;
        }
    }
    return false;
}

template<typename T, int MODE, int NT>
void launch_count(const dim3& g, const EsParams<T>& p, int64_t num_rows,
        int num_chan, int64_t chunk, int nc, const T* uvw, const T* freq,
        uint32_t* stable, uint32_t* gtable, hipStream_t stream)
{
    k_bucket_count<T, MODE, NT><<<g, NT, 0, stream>>>(p, num_rows, num_chan,
            chunk, nc, uvw, freq, stable, gtable);
}

// Both record levels: k_bucket_fill1 (chunk blocks) then k_bucket_fill2
// (super bin x chunk-group blocks).
template<typename T, int MODE, bool DO_W, int NT>
int launch_fill(int nc, int64_t chunk, const EsParams<T>& p,
        int64_t num_rows, int num_chan, const T* uvw, const T* freq,
        const T* vis, const T* weight, const BucketScratch* s,
        const uint32_t* stable, uint32_t* gtable, hipStream_t stream)
{
    const ScanBinsArgs sba{s->bin_start, s->item_start, s->totals,
            s->item_bin, s->item_capacity};
    k_bucket_fill1<T, MODE, DO_W, NT><<<nc + 1, NT, 0, stream>>>(p, num_rows,
            num_chan, chunk, uvw, freq, vis, weight, stable, s->bin_count,
            s->sb_start, (T*)s->recs1, sba);
    // Chunk groups x super bins: each block moves the records of one
    // group of kGroupChunks chunks of one super bin.
    const int ng = (nc + kGroupChunks - 1) / kGroupChunks;
    // Staged level 2 when blocks average a round or more of records.
    if (num_rows * num_chan >= (int64_t)kF2Round * ng * p.nsbins)
    {
        const size_t lds = fill2_lds_bytes<T, MODE, DO_W>(
                1 << (2 * p.sshift));
        if (lds > 64 * 1024)
        {
            const int e = allow_lds<k_bucket_fill2_staged<T, MODE, DO_W>>(
                    lds);
            if (e) return e;
        }
        k_bucket_fill2_staged<T, MODE, DO_W><<<dim3(ng, p.nsbins), 256, lds,
                stream>>>(p, nc, stable, gtable, s->bin_count, s->bin_start,
                s->sb_start, (const T*)s->recs1, (T*)s->recs);
        return 0;
    }
    k_bucket_fill2<T, MODE, DO_W><<<dim3(ng, p.nsbins), 256, 0, stream>>>(
            p, nc, stable, gtable, s->bin_count, s->bin_start, s->sb_start,
            (const T*)s->recs1, (T*)s->recs);
    return 0;
}

template<typename T>
int bucket(const EsParams<T>& p_in, Mode mode, int64_t num_rows, int num_chan,
        const T* uvw, const T* freq, const T* vis, const T* weight,
        BucketScratch* s, hipStream_t stream, uint32_t* n_entries,
        uint32_t* n_items)
{
    // 3-D: all w-planes at once (records keep pos_w, footprint()).
    EsParams<T> p = p_in;
    if (p.do_w) p.plane = -1;
    sdp_Error st = SDP_SUCCESS;
    sdp_Error* status = &st;
    const int64_t num_vis = num_rows * num_chan;
    const int nc = num_chunks(num_vis, p.tstride);
    const int64_t chunk = (num_rows + nc - 1) / nc;   // rows per chunk
    const int passes = (p.nbins + kBinsPerPass - 1) / kBinsPerPass;
    const dim3 grid_b((nc + kCountChunks - 1) / kCountChunks, passes);
    const int ng = (nc + kGroupChunks - 1) / kGroupChunks;
    // Group tile counts from the start of the table, chunk super-bin counts
    // from its end: for any two calls whose table needs fit the allocation
    // (need grows with nc, ng with nc) one's chunk rows never overlap the
    // other's group rows, so the group rows stay zero between calls (each
    // is cleared by its k_bucket_fill2 reader).
    uint32_t* gtable = s->table;                                   // [ng][nbins]
    uint32_t* stable = s->table + s->table_entries -
            (size_t)nc * p.nsbins;                                 // [nc][nsbins]
    if (p.nsbins < 1 || p.nsbins > kMaxSuperBins ||
            (1 << (2 * p.sshift)) > kMaxSuperTiles ||
            p.tstride != p.nbins + p.nsbins ||
            bucket_table_entries(nc, p.nbins, p.nsbins) > s->table_entries)
    {
        SDP_LOG_ERROR("Bucketing geometry / count table mismatch");
        return SDP_ERR_RUNTIME;
    }
    // The group rows of tile counts are accumulated atomically into a zeroed
    // table: zeroed here only after an allocation or an interrupted call.
    if (s->gtable_dirty)
        SDP_HIP_CHECK(hipMemsetAsync(s->table, 0, s->table_entries *
                sizeof(uint32_t), stream), status);
    if (*status) return *status;
    s->gtable_dirty = true;
    if (mode == MODE_GRID)
        launch_count<T, MODE_GRID, 1024>(grid_b, p, num_rows, num_chan,
                chunk, nc, uvw, freq, stable, gtable, stream);
    else
        launch_count<T, MODE_DEGRID, 1024>(grid_b, p, num_rows, num_chan,
                chunk, nc, uvw, freq, stable, gtable, stream);
    SDP_HIP_CHECK_LAUNCH(status);
    // Column prefixes (in place) and totals: tile counts over the chunk
    // groups into bin_count[0, nbins), super-bin counts over the chunks
    // into bin_count[nbins, nbins + nsbins).
    const int gblk = (p.nbins + 63) / 64, sblk = (p.nsbins + 63) / 64;
    k_scan_columns<<<gblk + sblk, 1024, 0, stream>>>(gtable, ng, p.nbins,
            s->bin_count, gblk, stable, nc, p.nsbins, s->bin_count + p.nbins);
    SDP_HIP_CHECK_LAUNCH(status);
    // No host round trip: records and work items are sized for the worst
    // case by the caller (BucketScratch::recs_bytes / item_capacity).
    const int words = (mode == MODE_GRID && p.do_w) ? 8 : 4;
    const size_t worst = (size_t)num_vis * (mode == MODE_GRID ? 4 : 1) *
            words * sizeof(T);
    if (worst > s->recs_bytes || (worst && !s->recs1))
    {
        SDP_LOG_ERROR("Bucketing scratch too small (%zu < %zu bytes)",
                s->recs_bytes, worst);
        return SDP_ERR_RUNTIME;
    }
    *n_entries = 0;                  // not known on the host
    *n_items = s->item_capacity;     // upper bound; extra items exit
    int fe;
    if (mode == MODE_GRID)
    {
        if (p.do_w)
            fe = launch_fill<T, MODE_GRID, true, 1024>(nc, chunk, p, num_rows,
                    num_chan, uvw, freq, vis, weight, s, stable, gtable,
                    stream);
        else
            fe = launch_fill<T, MODE_GRID, false, 1024>(nc, chunk, p,
                    num_rows, num_chan, uvw, freq, vis, weight, s, stable,
                    gtable, stream);
    }
    else
    {
        fe = launch_fill<T, MODE_DEGRID, false, 1024>(nc, chunk, p, num_rows,
                num_chan, uvw, freq, vis, weight, s, stable, gtable, stream);
    }
    SDP_HIP_CHECK((hipError_t)fe, status);
    SDP_HIP_CHECK_LAUNCH(status);
    if (!*status) s->gtable_dirty = false;
    return *status;
}

template<typename T>
int scatter(const EsParams<T>& p, const BucketScratch& s, uint32_t n_items,
        T* grid, hipStream_t stream, bool skip_empty, bool accumulate)
{
    sdp_Error st = SDP_SUCCESS;
    sdp_Error* status = &st;
    if (!accumulate)
    {
        k_zero_shared_tiles<T><<<p.nbins, kThreads, 0, stream>>>(
                p, s.item_start, grid);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    const int acc = accumulate ? 1 : 0;
    // f32: the matrix-core tile kernels with per-entry tap tables (float
    // plans have W <= 16, sdp_gridder_uvw_es_fft_utils.cpp:498); f64 (and
    // any wider float support): LDS accumulation below.
    if constexpr (sizeof(T) == 4)
    {
        const float* recs = (const float*)s.recs;
        const int se = (skip_empty ? 1 : 0) | (accumulate ? 2 : 0);
        if (p.support <= 16)
        {
            if (p.support <= 8 && p.do_w)
                k_scatter_tab<true, 9><<<n_items, 256, 0, stream>>>(
                        p, recs, s.bin_start, s.item_start, s.item_bin, grid,
                        se);
            else if (p.support <= 8)
                k_scatter_tab<false, 9><<<n_items, 256, 0, stream>>>(
                        p, recs, s.bin_start, s.item_start, s.item_bin, grid,
                        se);
            else if (p.do_w)
                k_scatter_tab<true, 17><<<n_items, 256, 0, stream>>>(
                        p, recs, s.bin_start, s.item_start, s.item_bin, grid,
                        se);
            else
                k_scatter_tab<false, 17><<<n_items, 256, 0, stream>>>(
                        p, recs, s.bin_start, s.item_start, s.item_bin, grid,
                        se);
            SDP_HIP_CHECK_LAUNCH(status);
            return *status;
        }
    }
    const size_t lds = 2 * (size_t)kTile * kScatterStride * sizeof(T);
    if (p.do_w)
    {
        SDP_HIP_CHECK(((hipError_t)allow_lds<k_scatter<T, true>>(lds)), status);
        k_scatter<T, true><<<n_items, kThreads, lds, stream>>>(
                p, (const T*)s.recs, s.bin_start, s.item_start, s.item_bin, grid,
                acc);
    }
    else
    {
        SDP_HIP_CHECK(((hipError_t)allow_lds<k_scatter<T, false>>(lds)), status);
        k_scatter<T, false><<<n_items, kThreads, lds, stream>>>(
                p, (const T*)s.recs, s.bin_start, s.item_start, s.item_bin, grid,
                acc);
    }
    SDP_HIP_CHECK_LAUNCH(status);
    return *status;
}

// 3-D, f32, W <= 8: w-planes p.plane .. p.plane + nplanes - 1 (into
// grids[0..nplanes)) in one pass of the tile kernel (k_scatter_tab<.., 2 or
// 3>): the staging, visit lists and operand reads of the entries are shared
// by the planes.
template<typename T>
int planes_per_pass(const EsParams<T>& p)
{
    return (sizeof(T) == 4 && p.do_w && p.support <= 8) ? kScatterPlanes : 1;
}

template<typename T>
int scatter_planes(const EsParams<T>& p, const BucketScratch& s,
        uint32_t n_items, T* const* grids, int nplanes, hipStream_t stream,
        bool skip_empty)
{
    sdp_Error st = SDP_SUCCESS;
    sdp_Error* status = &st;
    if (nplanes < 2 || nplanes > planes_per_pass(p)) return SDP_ERR_RUNTIME;
    if constexpr (sizeof(T) == 4)
    {
        for (int q = 0; q < nplanes; ++q)
        {
            k_zero_shared_tiles<T><<<p.nbins, kThreads, 0, stream>>>(
                    p, s.item_start, grids[q]);
            SDP_HIP_CHECK_LAUNCH(status);
        }
        const int se = skip_empty ? 1 : 0;
        const float* recs = (const float*)s.recs;
        static_assert(kScatterPlanes == 2, "one multi-plane kernel");
        k_scatter_tab<true, 9, kScatterChunk, kScatterPlanes><<<n_items, 256,
                0, stream>>>(p, recs, s.bin_start, s.item_start, s.item_bin,
                grids[0], se, grids[1], p.plane + 1);
        SDP_HIP_CHECK_LAUNCH(status);
    }
    return *status;
}

// f32: W <= 8 the lane-per-entry window gather (k_gather_win), W = 16 the
// matrix-core sub-tile form (k_gather_tab); f64: the LDS window gather.
template<typename T>
int gather(const EsParams<T>& p, const BucketScratch& s, uint32_t n_items,
        const T* grid, T* vis, hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    sdp_Error* status = &st;
    if constexpr (sizeof(T) == 4)
    {
        const float* recs = (const float*)s.recs;
        if (p.support <= 16)
        {
            if (p.support <= 8)
            {
                // Lane-per-entry window gather (no record sort needed).
                // Half-tile windows (40 x 72: twice the workgroups per CU
                // as the 72 x 72 window, 0.52 -> 0.46 ms at config 2).
                constexpr int kR = 32, kNT = 256;
                const uint32_t nb = n_items * (kTile / kR);
                if (p.do_w)
                    k_gather_win<true, 9, kR, kNT><<<nb, kNT, 0, stream>>>(
                            p, recs, s.bin_start, s.item_start, s.item_bin,
                            grid, vis);
                else
                    k_gather_win<false, 9, kR, kNT><<<nb, kNT, 0, stream>>>(
                            p, recs, s.bin_start, s.item_start, s.item_bin,
                            grid, vis);
                SDP_HIP_CHECK_LAUNCH(status);
                return *status;
            }
            if (p.do_w)
                k_gather_tab<true, 17><<<n_items, 256, 0, stream>>>(p, recs,
                        s.bin_start, s.item_start, s.item_bin, grid, vis);
            else
                k_gather_tab<false, 17><<<n_items, 256, 0, stream>>>(p, recs,
                        s.bin_start, s.item_start, s.item_bin, grid, vis);
            SDP_HIP_CHECK_LAUNCH(status);
            return *status;
        }
    }
    const int wrows = kTile + p.support;
    int ws = wrows;
    while (ws % 32 != 8 && ws % 32 != 24) ++ws;
    const size_t lds = 2 * (size_t)wrows * ws * sizeof(T);
    if (lds > 160 * 1024)
    {
        SDP_LOG_ERROR("Support %d too large for the LDS window", p.support);
        return SDP_ERR_INVALID_ARGUMENT;
    }
    if (p.do_w)
    {
        SDP_HIP_CHECK(((hipError_t)allow_lds<k_gather<T, true>>(lds)), status);
        k_gather<T, true><<<n_items, kThreads, lds, stream>>>(p,
                (const T*)s.recs, s.bin_start, s.item_start, s.item_bin, grid,
                vis, wrows, ws);
    }
    else
    {
        SDP_HIP_CHECK(((hipError_t)allow_lds<k_gather<T, false>>(lds)), status);
        k_gather<T, false><<<n_items, kThreads, lds, stream>>>(p,
                (const T*)s.recs, s.bin_start, s.item_start, s.item_bin, grid,
                vis, wrows, ws);
    }
    SDP_HIP_CHECK_LAUNCH(status);
    return *status;
}

template<typename T>
int screen_corr_2d(const ImageParams<T>& ip, const T* layer, T* dirty,
        hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    k_screen_corr_2d<T><<<image_blocks(ip.N), dim3(64, 4), 0, stream>>>(
            ip, layer, dirty);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<typename T>
int screen_accumulate(const ImageParams<T>& ip, int plane, const T* layer,
        T* dirty, hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    k_screen_accumulate<T><<<image_blocks(ip.N), dim3(64, 4), 0, stream>>>(
            ip, plane, layer, dirty);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<typename T>
int apply_correction(const ImageParams<T>& ip, T* dirty, hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    k_apply_correction<T><<<image_blocks(ip.N / 2 + 1), dim3(64, 4), 0,
            stream>>>(ip, dirty);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<typename T>
int reverse_screen(const ImageParams<T>& ip, int plane, T* dirty,
        bool correct_in_place, T* grid, hipStream_t stream)
{
    sdp_Error st = SDP_SUCCESS;
    k_reverse_screen<T><<<image_blocks(ip.G), dim3(64, 4), 0, stream>>>(
            ip, plane, dirty, correct_in_place ? 1 : 0, grid);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

#define SDP_ES_INSTANTIATE(T) \
    template int bucket<T>(const EsParams<T>&, Mode, int64_t, int, const T*, \
            const T*, const T*, const T*, BucketScratch*, hipStream_t, \
            uint32_t*, uint32_t*); \
    template int scatter<T>(const EsParams<T>&, const BucketScratch&, \
            uint32_t, T*, hipStream_t, bool, bool); \
    template int planes_per_pass<T>(const EsParams<T>&); \
    template int scatter_planes<T>(const EsParams<T>&, \
            const BucketScratch&, uint32_t, T* const*, int, hipStream_t, \
            bool); \
    template int gather<T>(const EsParams<T>&, const BucketScratch&, \
            uint32_t, const T*, T*, hipStream_t); \
    template int screen_corr_2d<T>(const ImageParams<T>&, const T*, T*, \
            hipStream_t); \
    template int screen_accumulate<T>(const ImageParams<T>&, int, const T*, \
            T*, hipStream_t); \
    template int apply_correction<T>(const ImageParams<T>&, T*, hipStream_t); \
    template int reverse_screen<T>(const ImageParams<T>&, int, T*, bool, T*, \
            hipStream_t);

SDP_ES_INSTANTIATE(float)
SDP_ES_INSTANTIATE(double)

} // namespace sdp_es
