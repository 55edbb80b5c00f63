// MI355X-native dynamic-threshold RFI flagger.
//
// Replaces src/ska-sdp-func/visibility/sdp_flagger.cpp (ska-sdp-func 1.2.2)
// with bit-identical results. The reference walks every (baseline, pol)
// stream sequentially in time with 3-4 qsorts of <= num_channels doubles
// per step (:125-339). Here one 64-lane wave owns a stream: the channels of
// a time step live in registers (channel c in lane c % 64, slot c / 64),
// and every median is an exact order statistic selected on the IEEE bit
// patterns (all the values ranked are >= 0, so bit-pattern order is value
// order). Each statistic is bracketed by its value at the previous time
// step: one counting pass (compare + ballot + popcount per register) checks
// that the bracket holds the k-th key and compacts the ~64 keys inside it
// into LDS, and radix rounds over those two registers (an LDS histogram of
// 64 digit ranges and a cross-lane scan per round) finish it -- no sort. A
// bracket miss falls back to a bitwise search over all keys, so the result
// never depends on the bracket. The stream state (previous
// magnitudes, transit scores) stays in registers across time steps; the
// median history is a per-wave LDS ring; window flagging reads trigger
// bytes from LDS. Flags are written only where set (idempotent stores of
// 1), so the output keeps whatever the caller's array held.
#include <cmath>
#include <cstdio>
#include <cstdint>
#include <cstring>

#include "ska-sdp-func/visibility/sdp_flagger.h"
#include "../utility/sdp_hip.h"

namespace {

constexpr int kWaves = 4;                 // streams per workgroup
constexpr int kMaxChannels = 2048;        // 32 registers per lane
constexpr int kMaxHistory = 1024;

struct FlagParams
{
    int64_t T, B;
    int C, P;
    int ns;          // number of sampled channels, C / step (:145)
    int step;
    int window;
    int wmh;         // window_median_history
    double alpha, thr_mag, thr_var, thr_bb;
};

// |v| exactly as the reference's std::abs(std::complex<FP>) on glibc:
// cabsf(z) = hypotf, computed in double and rounded once to float;
// cabs(z) = glibc's hypot (its non-FMA kernel, sysdeps/ieee754/dbl-64
// e_hypot.c of glibc 2.35). Both reproduced operation for operation.

__device__ __forceinline__ double mag_of(float re, float im)
{
#pragma clang fp contract(off)
    const double x = (double)re, y = (double)im;
    return (double)(float)sqrt(x * x + y * y);
}

__device__ __forceinline__ double hypot_kernel(double ax, double ay)
{
#pragma clang fp contract(off)
    double h = sqrt(ax * ax + ay * ay);
    double t1, t2;
    if (h <= 2.0 * ay)
    {
        const double delta = h - ay;
        t1 = ax * (2.0 * delta - ax);
        t2 = (delta - 2.0 * (ax - ay)) * delta;
    }
    else
    {
        const double delta = h - ax;
        t1 = 2.0 * delta * (ax - 2.0 * ay);
        t2 = (4.0 * delta - ay) * ay + delta * delta;
    }
    h -= (t1 + t2) / (2.0 * h);
    return h;
}

__device__ __forceinline__ double mag_of(double re, double im)
{
#pragma clang fp contract(off)
    const double x = fabs(re), y = fabs(im);
    if (!isfinite(x) || !isfinite(y))
        return (isinf(x) || isinf(y)) ? INFINITY : x + y;
    const double ax = x < y ? y : x;
    const double ay = x < y ? x : y;
    constexpr double kScale = 0x1p-600, kLarge = 0x1p+511;
    constexpr double kTiny = 0x1p-511, kEps = 0x1p-54;
    if (ax > kLarge)
    {
        if (ay <= ax * kEps) return ax + ay;
        return hypot_kernel(ax * kScale, ay * kScale) / kScale;
    }
    if (ay < kTiny)
    {
        if (ax >= ay / kEps) return ax + ay;
        return hypot_kernel(ax / kScale, ay / kScale) * kScale;
    }
    if (ay <= ax * kEps) return ax + ay;
    return hypot_kernel(ax, ay);
}

// sorted[round(0.5 n)] (:83-88); n == 1 reads sorted[0] (the reference reads
// one past the end there, at t == 0 only, where the value is discarded).
__device__ __forceinline__ int mid_index(int n)
{
    const int m = (n + 1) / 2;
    return m < n ? m : n - 1;
}

// ---------------------------------------------------------------------------
// Exact order statistics over a wave.
//
// Every value ranked is >= 0, so the IEEE bit pattern orders like the value:
// a statistic is selected on integer keys (float -> 32-bit, double -> 64-bit
// patterns). Elements that do not take part carry the key ~0 (above every
// non-negative pattern, NaNs included), so counting needs no masks.
//
// search() is a bitwise binary search for the k-th smallest key inside an
// interval [L, U) known to hold it (c0 = #(key < L) <= k < c1 = #(key < U)).
// Each probe costs one compare + ballot + popcount per register; probes that
// fall outside (L, U) are decided without counting, and the search ends as
// soon as the interval holds a single key, which is then read out directly.
//
// select_tracked() brackets each statistic by the previous time step's value
// (x +- w per statistic and stream): one pass counts the keys below and inside
// the bracket and compacts the inside ones into LDS; if the k-th key is inside
// and the bracket holds <= 64 R keys, radix_select() runs on R registers of
// candidates instead of all of them. A miss falls back to the search over all
// keys (still exact); w adapts so that the bracket holds ~32 R candidates.
// Results never depend on the bracket -- only the cost does.
// ---------------------------------------------------------------------------
template<typename V> struct KeyOf;
template<> struct KeyOf<float>
{
    using type = uint32_t;
    static constexpr int kTop = 30;     // highest bit of a non-negative key
};
template<> struct KeyOf<double>
{
    using type = uint64_t;
    static constexpr int kTop = 62;
};

__device__ __forceinline__ uint32_t key_of(float v) { return __float_as_uint(v); }
__device__ __forceinline__ uint64_t key_of(double v)
{
    return (uint64_t)__double_as_longlong(v);
}
__device__ __forceinline__ float val_of(uint32_t k) { return __uint_as_float(k); }
__device__ __forceinline__ double val_of(uint64_t k)
{
    return __longlong_as_double((long long)k);
}

__device__ __forceinline__ uint64_t ballot(bool p)
{
    return __builtin_amdgcn_ballot_w64(p);
}

__device__ __forceinline__ uint32_t readlane(uint32_t v, int lane)
{
    return (uint32_t)__builtin_amdgcn_readlane((int)v, lane);
}
__device__ __forceinline__ uint64_t readlane(uint64_t v, int lane)
{
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readlane((int)(uint32_t)v,
            lane);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readlane(
            (int)(uint32_t)(v >> 32), lane);
    return ((uint64_t)hi << 32) | lo;
}

// flags[row + (lane + 64 j) P] = 1 as a uniform row base (scalar) plus one
// 32-bit per-lane offset, so no per-element address stays live.
__device__ __forceinline__ void set_flag(int32_t* row, int j, int P, int lane)
{
    char* base = (char*)(row + 64 * j * P);
    *(int32_t*)(base + (uint32_t)(lane * P) * 4u) = 1;
}


// Key sets: key(j), j < N, from a register array or computed on the fly
// (a statistic's keys are then never held as an array: they are rebuilt in
// the bracket pass and, rarely, in the full search).
template<typename K, int N>
struct ArrayKeys
{
    const K (&a)[N];
    __device__ __forceinline__ K operator()(int j) const { return a[j]; }
};

template<typename K, int N, class Keys>
__device__ __forceinline__ int count_lt(const Keys& key, K c)
{
    int s = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) s += __popcll(ballot(key(j) < c));
    return s;
}

// CHECKS: decide probes outside (L, U) without counting (worth it over all
// keys). Without it L and U are implied by prefix and bit, which holds
// when the set lies inside [prefix, prefix + 2^(bit+1)) -- true of the
// compacted bracket candidates -- and a probe is one counting pass.
template<typename K, int N, bool CHECKS, class Keys>
__device__ __forceinline__ K search(const Keys& key, int k, K prefix,
        int bit, K L, K U, int c0, int c1, int& nprobe)
{
    while (c1 - c0 > 1 && bit >= 0)
    {
        const K cand = prefix | ((K)1 << bit);
        if (CHECKS && cand <= L)
        {
            prefix = cand;
        }
        else if (!CHECKS || cand < U)
        {
            const int cnt = count_lt<K, N>(key, cand);
            ++nprobe;
            if (cnt <= k)
            {
                prefix = cand;
                if (CHECKS) L = cand;
                c0 = cnt;
            }
            else
            {
                if (CHECKS) U = cand;
                c1 = cnt;
            }
        }
        --bit;
    }
    if (c1 - c0 > 1) return prefix;        // every bit decided: ties
    if (!CHECKS)
    {
        L = prefix;
        U = prefix + (bit >= 0 ? (K)2 << bit : (K)1);
    }
    K ans = L;                             // the one key in [L, U)
#pragma unroll
    for (int j = 0; j < N; ++j)
    {
        const K kj = key(j);
        const uint64_t m = ballot(kj >= L) & ballot(kj < U);
        if (m) ans = readlane(kj, (int)__builtin_ctzll(m));
    }
    return ans;
}

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
}

// Inclusive prefix sum over the 64 lanes: DPP row shifts inside rows of
// 16, then the row broadcasts (no LDS round trips).
__device__ __forceinline__ uint32_t wave_incl_scan(uint32_t x)
{
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x111, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x112, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x114, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x118, 0xf, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x142, 0xa, 0xf, false);
    x += (uint32_t)__builtin_amdgcn_update_dpp(0, (int)x, 0x143, 0xc, 0xf, false);
    return x;
}

// Radix rounds for the k-th smallest of the n keys inside [L, U) (keys
// outside it do not take part). A round splits [L, U) into 64 digit
// ranges of 2^shift keys, counts the keys of each in an LDS histogram
// (one ds_add per register), scans the 64 counts across the lanes and
// keeps the digit range that holds the k-th key: ~6 key bits per round,
// ~30 instructions, against one compare + ballot + popcount probe per bit
// of the bitwise search. Ends when the range holds a single key (read out)
// or a single value (ties). bins: 64 words of LDS. The caller guarantees
// that [L, U) holds the k-th key; if a round finds no digit range past k
// (the guarantee broken) ok is cleared and the caller falls back to the
// search over every key, instead of reading lane 64 of a zero ballot.
template<typename K, int N, class Keys>
__device__ __forceinline__ K radix_select(const Keys& key, int k, K L, K U,
        int n, uint32_t* bins, int lane, int& nround, bool& ok)
{
    ok = true;
    while (n > 1 && U - L > 1)
    {
        const K span = U - L;
        const int len = (int)(8 * sizeof(K)) - (sizeof(K) == 8 ?
                __clzll((long long)(span - 1)) : __clz((int)(span - 1)));
        const int shift = len > 6 ? len - 6 : 0;
        bins[lane] = 0u;
        wave_sync();
#pragma unroll
        for (int j = 0; j < N; ++j)
        {
            const K d = key(j) - L;
            if (d < span)
                __hip_atomic_fetch_add(&bins[(uint32_t)(d >> shift)], 1u,
                        __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        }
        wave_sync();
        const uint32_t cnt = bins[lane];
        const uint32_t incl = wave_incl_scan(cnt);
        const uint64_t over = __builtin_amdgcn_ballot_w64(incl > (uint32_t)k);
        if (over == 0)
        {
            ok = false;
            wave_sync();
            return L;
        }
        const int b = (int)__builtin_ctzll(over);
        k -= (int)__builtin_amdgcn_readlane((int)(incl - cnt), b);
        n = __builtin_amdgcn_readlane((int)cnt, b);
        L += (K)b << shift;
        const K top = L + ((K)1 << shift);
        if (top < U) U = top;
        ++nround;
        wave_sync();
    }
    if (n > 1 || U - L <= 1) return L;      // one value left (ties)
    K ans = L;                              // the one key in [L, U)
#pragma unroll
    for (int j = 0; j < N; ++j)
    {
        const K kj = key(j);
        const uint64_t m = ballot(kj - L < U - L);
        if (m) ans = readlane(kj, (int)__builtin_ctzll(m));
    }
    return ans;
}

// Wave-uniform double in scalar registers.
__device__ __forceinline__ double uniform(double x)
{
    const uint64_t b = (uint64_t)__double_as_longlong(x);
    const uint32_t lo = (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    const uint32_t hi = (uint32_t)__builtin_amdgcn_readfirstlane(
            (int)(uint32_t)(b >> 32));
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}

#ifdef SDP_FLAGGER_STATS
// Per statistic: [init, hit (compacted), hit (all keys), miss, probes over
// candidates, probes over all keys, hit at the second bracket].
__device__ unsigned long long g_flag_stats[6][7];
#endif

struct Track
{
    double x, w;     // previous value, bracket half-width
    bool valid;
};

template<typename V, int N, int R, class Keys>
__device__ __forceinline__ V select_tracked(const Keys& key, int k,
        int nvalid, Track& tr, typename KeyOf<V>::type* cand_lds, int lane,
        int sid)
{
    using K = typename KeyOf<V>::type;
    constexpr int kTop = KeyOf<V>::kTop;
    constexpr K kSpan = (K)1 << (kTop + 1);
    constexpr bool kCompact = N > R;
    constexpr int kCap = 64 * R;
    // Search set: all keys, or the compacted bracket candidates.
    K prefix = 0, L = 0, U = kSpan;
    int bit = kTop, c0 = 0, c1 = nvalid, kk = k, n_in = 0, attempt = 0;
    bool hit = false, use_cand = false;
    if (tr.valid)
    {
        // Attempt 0: the bracket x +- w. On a miss, attempt 1 looks 4 w
        // further on the side of the miss before falling back to the search
        // over every key (which starts from the interval the misses left).
        double lo_d = tr.x - tr.w, hi_d = tr.x + tr.w;
#pragma unroll 1
        for (; attempt < 2; ++attempt)
        {
            V lo_v = (V)lo_d;
            if (!(lo_v > (V)0)) lo_v = (V)0;
            K lo = key_of(lo_v), hi = key_of((V)hi_d);
            if (!(hi < kSpan)) hi = kSpan - 1;
            if (lo < L) lo = L;
            if (hi > U - 1) hi = U - 1;
            if (lo > hi) break;
            // One pass: count the keys below the bracket and compact the
            // ones inside it (positions past the capacity all land on the
            // spare slot kCap, so the store needs no branch).
            int c_lt = 0;
            n_in = 0;
#pragma unroll
            for (int j = 0; j < N; ++j)
            {
                const K kj = key(j);
                const uint64_t mb = ballot(kj < lo);
                const uint64_t mi = ballot(kj <= hi) & ~mb;
                if (kCompact)
                {
                    const uint32_t pos = __builtin_amdgcn_mbcnt_hi(
                            (uint32_t)(mi >> 32), __builtin_amdgcn_mbcnt_lo(
                            (uint32_t)mi, (uint32_t)n_in));
                    const bool inside = __builtin_amdgcn_inverse_ballot_w64(mi);
                    cand_lds[inside && pos < (uint32_t)kCap ? pos : kCap] = kj;
                }
                c_lt += __popcll(mb);
                n_in += __popcll(mi);
            }
            if (c_lt <= k && k < c_lt + n_in)
            {
                hit = true;
                L = lo;
                U = hi + 1;
                c0 = c_lt;
                c1 = c_lt + n_in;
                if (lo == hi)
                {
                    prefix = lo;
                    bit = -1;
                }
                else
                {
                    bit = (int)(8 * sizeof(K)) - 1 -
                            (sizeof(K) == 8 ? __clzll((long long)(lo ^ hi)) :
                                              __clz((int)(lo ^ hi)));
                    prefix = lo & ~(((K)2 << bit) - 1);
                }
                if (kCompact && n_in <= kCap)
                {
                    use_cand = true;
                    kk = k - c_lt;
                    c0 = 0;
                    c1 = n_in;
                }
                break;
            }
            if (k < c_lt)
            {
                U = lo;
                c1 = c_lt;
                hi_d = lo_d;
                lo_d = lo_d - 4.0 * tr.w;
            }
            else
            {
                L = hi + 1;
                c0 = c_lt + n_in;
                lo_d = hi_d;
                hi_d = hi_d + 4.0 * tr.w;
            }
        }
    }
    int nprobe = 0;
    K ans;
    bool ok = true;
    if (hit && (use_cand || !kCompact))
    {
        // The bracket holds the k-th key: radix rounds over the compacted
        // candidates (or, N <= R, over the keys themselves).
        uint32_t* bins = (uint32_t*)(cand_lds + kCap + 2);
        if (kCompact)
        {
            wave_sync();
            K c[kCompact ? R : 1];
#pragma unroll
            for (int r = 0; r < (kCompact ? R : 1); ++r)
            {
                const int s = lane + 64 * r;
                c[r] = s < n_in ? cand_lds[s] : ~(K)0;
            }
            ans = radix_select<K, kCompact ? R : 1>(
                    ArrayKeys<K, kCompact ? R : 1>{c}, kk, L, U, n_in, bins,
                    lane, nprobe, ok);
        }
        else
        {
            ans = radix_select<K, N>(key, kk - c0, L, U, c1 - c0, bins,
                    lane, nprobe, ok);
        }
        wave_sync();
        if (!ok)   // bracket bookkeeping broken: search every key
            ans = search<K, N, true>(key, k, (K)0, kTop, (K)0, kSpan, 0,
                    nvalid, nprobe);
    }
    else
    {
        ans = search<K, N, true>(key, kk, prefix, bit, L, U, c0, c1,
                nprobe);
    }

    // Bracket for the next time step: centred on this value, half-width
    // scaled so the bracket holds about `target` keys.
#ifdef SDP_FLAGGER_STATS
    if (lane == 0)
    {
        const int cls = !tr.valid ? 0 : (!hit ? 3 : (attempt > 0 ? 6 :
                (use_cand ? 1 : 2)));
        atomicAdd(&g_flag_stats[sid][cls], 1ull);
        atomicAdd(&g_flag_stats[sid][use_cand ? 4 : 5],
                (unsigned long long)nprobe);
    }
#endif
    const double a = (double)val_of(ans);
    // The width factor only steers the cost: single precision with the
    // hardware reciprocal (a double division here was ~12 instructions per
    // selection, 6 selections per step).
    const float target = fminf(32.0f * R, fmaxf(1.0f, 0.125f * nvalid));
    const float inv_in = __builtin_amdgcn_rcpf((float)(n_in > 1 ? n_in : 1));
    if (!tr.valid)
    {
        tr.w = a * 0x1p-7;
    }
    else if (hit && attempt == 0)
    {
        float f = target * inv_in;
        if (n_in <= kCap) f = f < 0.5f ? 0.5f : (f > 2.0f ? 2.0f : f);
        tr.w *= (double)f;
    }
    else if (hit)
    {
        // Found one step beyond the bracket (a 4 w wide window): widen.
        const float f = 2.0f * target * inv_in;
        tr.w *= (double)(f < 1.0f ? 1.0f : (f > 2.0f ? 2.0f : f));
    }
    else if (!(tr.w > 0.0))
    {
        const double d = fabs(a - tr.x);
        tr.w = (d > 0.0) ? d : a * 0x1p-10;
    }
    if (!(tr.w <= fabs(a) * 1024.0)) tr.w = fabs(a) * 1024.0;
    if (!(tr.w >= 0.0)) tr.w = 0.0;
    tr.x = a;
    tr.w = uniform(tr.w);         // bracket state stays in scalar registers
    tr.valid = isfinite(a);
    return val_of(ans);
}

// (:104-122)
__device__ __forceinline__ double modified_zscore(double median,
        double mediandev, double val)
{
#pragma clang fp contract(off)
    if (mediandev == 0 && val == median) return 0.0;
    if (mediandev == 0 && val != median) return 10000000.0;
    return 0.6795 * (val - median) / mediandev;
}

// modified_zscore compared with a threshold:
// z > thr || z < -thr  <=>  |z| > thr (for every thr, NaNs included).
// The division is replaced by a multiply with the reciprocal wherever that
// cannot change the outcome: |q - z| <= 2^-50 |z| for normal divisors, so
// only values within 2^-44 thr of the threshold take the exact division.
struct ZTest
{
    double med, dev, inv, thr, band;
    bool dev0, fast;
};

__device__ __forceinline__ ZTest make_ztest(double med, double dev,
        double thr)
{
    ZTest z;
    z.med = med;
    z.dev = dev;
    z.thr = thr;
    z.dev0 = (dev == 0);
    const double adev = fabs(dev);
    z.fast = adev > 0x1p-1000 && adev < 0x1p+1000 &&
            thr > 0x1p-900 && thr < 0x1p+900;
    z.inv = z.fast ? 1.0 / dev : 0.0;
    z.band = thr * 0x1p-44;
    return z;
}

__device__ __forceinline__ bool z_exceeds(const ZTest& zt, double val)
{
#pragma clang fp contract(off)
    if (zt.dev0)
    {
        const double z = (val == zt.med) ? 0.0 : 10000000.0;
        return z > zt.thr || z < -zt.thr;
    }
    const double num = 0.6795 * (val - zt.med);
    if (zt.fast)
    {
        const double aq = fabs(num * zt.inv);
        if (!(fabs(aq - zt.thr) <= zt.band)) return aq > zt.thr;
    }
    const double z = num / zt.dev;
    return z > zt.thr || z < -zt.thr;
}

// z_exceeds for the EPL register slots of a lane at once, as bit j of the
// result. The reciprocal test runs branch-free on every slot; only when some
// lane's slot falls inside the exact-division band (or the test has no fast
// form) does the whole wave redo the slots with z_exceeds, which gives the
// same bits (outside the band the two agree). Per-slot divergent branches
// cost ~40 scalar / exec-mask instructions each.
template<int EPL, class Val>
__device__ __forceinline__ uint32_t z_bits(const ZTest& zt, const Val& val)
{
#pragma clang fp contract(off)
    uint32_t bits = 0;
    bool exact = zt.dev0 || !zt.fast;
    if (!exact)
    {
        bool unsure = false;
#pragma unroll
        for (int j = 0; j < EPL; ++j)
        {
            const double aq = fabs(0.6795 * (val(j) - zt.med) * zt.inv);
            bits |= (aq > zt.thr ? 1u : 0u) << j;
            unsure = unsure || fabs(aq - zt.thr) <= zt.band;
        }
        exact = __builtin_amdgcn_ballot_w64(unsure) != 0;
    }
    if (exact)
    {
        bits = 0;
#pragma unroll
        for (int j = 0; j < EPL; ++j)
            bits |= (z_exceeds(zt, val(j)) ? 1u : 0u) << j;
    }
    return bits;
}

// Window spread (:224-240, :316-337): channel d is flagged if it triggered,
// or a trigger sits i <= window channels above it and d > 0, or i <= window
// channels below it.
__device__ __forceinline__ bool spread(const uint8_t* trig, int d, int C,
        int window)
{
    bool f = trig[d] != 0;
    for (int i = 1; i <= window; ++i)
    {
        if (d > 0 && d + i < C && trig[d + i]) f = true;
        if (d - i >= 0 && trig[d - i]) f = true;
    }
    return f;
}

// Occupancy: the float kernels fit 128 VGPRs (4 waves per SIMD) with a few
// dwords of spill, which measures faster than 3 waves without; the double
// kernels (two registers per statistic key) stay at 3. Two candidate
// registers (128 keys) measured faster than one, three or four.
#define FLAGGER_WAVES \
    __attribute__((amdgpu_waves_per_eu(sizeof(FP) == 4 ? 4 : 3)))
constexpr int kCandRegs = 2;   // compacted candidates: 64 per register

// Per-wave LDS layout: median history | trigger bytes (all, variation) |
// candidate keys | radix-round histogram.
__host__ __device__ inline size_t lds_per_wave(int wmh, int C)
{
    return (size_t)wmh * 8 + 2 * (size_t)((C + 15) & ~15) +
            (64 * kCandRegs + 2) * 8 + 68 * 4;
}

// FULL: sampling_step 1 and C == 64 EPL, so every register slot is a sampled
// channel and the magnitude / transit arrays are their own keys.
template<typename FP, int EPL, int HEPL, bool FULL>
__global__ __launch_bounds__(64 * kWaves) FLAGGER_WAVES void k_flagger(
        const FP* __restrict__ vis, int32_t* __restrict__ flags,
        FlagParams prm)
{
#pragma clang fp contract(off)
    using KM = typename KeyOf<FP>::type;
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane0 = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t stream = (int64_t)blockIdx.x * kWaves + wave;
    if (stream >= prm.B * prm.P) return;   // whole wave
    const int64_t b = stream / prm.P;
    const int p = (int)(stream % prm.P);
    const int C = prm.C;
    const int cpad = (C + 15) & ~15;
    unsigned char* base = smem + lds_per_wave(prm.wmh, C) * wave;
    double* hist = (double*)base;
    uint8_t* trig_all = base + (size_t)prm.wmh * 8;
    uint8_t* trig_var = trig_all + cpad;
    void* cand = trig_var + cpad;
    const int k_s = mid_index(prm.ns);

    bool ch_ok[EPL], smp_ok[EPL];
    uint32_t ok_bits = 0;          // bit j: ch_ok[j]
#pragma unroll
    for (int j = 0; j < EPL; ++j)
    {
        const int c = lane0 + 64 * j;
        ch_ok[j] = FULL || c < C;
        ok_bits |= (ch_ok[j] ? 1u : 0u) << j;
        smp_ok[j] = FULL || (c < C && (c % prm.step) == 0 &&
                (c / prm.step) < prm.ns);
    }
    FP m[EPL], prev[EPL];
    double transit[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j)
    {
        prev[j] = (FP)0;
        transit[j] = 0.0;
    }
    Track tk_mag{0, 0, false}, tk_dev{0, 0, false};
    Track tk_var{0, 0, false}, tk_vdev{0, 0, false};
    Track tk_h{0, 0, false}, tk_hdev{0, 0, false};

    const int64_t time_block = prm.B * (int64_t)C * prm.P;
    const int64_t stream_off = b * (int64_t)C * prm.P + p;
    // One complex value per register slot. Latency is hidden by occupancy
    // (4 streams per SIMD) rather than by a register prefetch of the next
    // step, which would cost 32 registers and a wave per SIMD.
    typedef FP FP2 __attribute__((ext_vector_type(2)));
    FP2 raw[EPL];
    auto load_step = [&](int64_t tt, int P, int lane) {
        const FP* vrow = vis + 2 * (tt * time_block + stream_off);
#pragma unroll
        for (int j = 0; j < EPL; ++j)
        {
            if (ch_ok[j])
            {
                const char* zb = (const char*)(vrow + 128 * j * P);
                raw[j] = *(const FP2*)(zb + (uint32_t)(lane * P) *
                        (2 * sizeof(FP)));
            }
        }
    };
    double prev_median = 0.0;
    int hpos = 0;                   // t % wmh, the ring slot of step t
    for (int64_t t = 0; t < prm.T; ++t)
    {
        // Opaque per step, so that the per-element address and LDS offset
        // arithmetic is not hoisted out of the time loop as dozens of
        // loop-invariant registers.
        int P = prm.P, lane = lane0;
        asm volatile("" : "+s"(P));
        asm volatile("" : "+v"(lane));
        const int64_t row = t * time_block + stream_off;
        int32_t* frow = flags + row;
        int32_t* fprev = frow - time_block;
        load_step(t, P, lane);
#pragma unroll
        for (int j = 0; j < EPL; ++j)
            m[j] = ch_ok[j] ? (FP)mag_of(raw[j].x, raw[j].y) : (FP)0;
        // Transit update first (:262-274), so the previous magnitudes are
        // dead before the selections and share registers with m.
        if (t > 0)
        {
#pragma unroll
            for (int j = 0; j < EPL; ++j)
            {
                const double rate = fabs((double)prev[j] - (double)m[j]);
                transit[j] = (t == 1) ? rate :
                        prm.alpha * rate + (1 - prm.alpha) * transit[j];
            }
        }

        // Magnitude median and MAD over the sampled channels (:170-178).
        double median, mediandev;
        {
            auto km = [&](int j) -> KM {
                return smp_ok[j] ? key_of(m[j]) : ~(KM)0;
            };
            median = (double)select_tracked<FP, EPL, kCandRegs>(km, k_s,
                    prm.ns, tk_mag, (KM*)cand, lane, 0);
        }
        {
            // |m - median| keys, rebuilt wherever they are read.
            auto kd = [&](int j) -> uint64_t {
                return smp_ok[j] ? key_of(fabs((double)m[j] - median)) :
                                   ~(uint64_t)0;
            };
            mediandev = select_tracked<double, EPL, kCandRegs>(kd, k_s,
                    prm.ns, tk_dev, (uint64_t*)cand, lane, 1);
        }

        // Broadband: median history of the last min(t + 1, wmh) steps.
        if (lane == 0) hist[hpos] = median;
        wave_sync();
        const int medwindow = (int)((t + 1 < prm.wmh) ? t + 1 : prm.wmh);
        bool situation = false;
        if (t != 0)
        {
            double hv[HEPL];
            uint64_t hk[HEPL];
#pragma unroll
            for (int j = 0; j < HEPL; ++j)
            {
                const int tt = lane + 64 * j;
                const bool ok = tt < medwindow;
                // Ring slot of step t - tt (tt < wmh): no 64-bit modulo.
                const int slot = hpos - tt < 0 ? hpos - tt + prm.wmh :
                                                 hpos - tt;
                hv[j] = ok ? hist[slot] : 0.0;
                hk[j] = ok ? key_of(hv[j]) : ~(uint64_t)0;
            }
            const int k_h = mid_index(medwindow);
            const double medmed = select_tracked<double, HEPL, kCandRegs>(
                    ArrayKeys<uint64_t, HEPL>{hk}, k_h, medwindow, tk_h,
                    (uint64_t*)cand, lane, 2);
#pragma unroll
            for (int j = 0; j < HEPL; ++j)
            {
                if (hk[j] != ~(uint64_t)0) hk[j] = key_of(fabs(hv[j] - medmed));
            }
            const double medmeddev = select_tracked<double, HEPL, kCandRegs>(
                    ArrayKeys<uint64_t, HEPL>{hk}, k_h, medwindow, tk_hdev,
                    (uint64_t*)cand, lane, 3);
            const double zmed = modified_zscore(medmed, medmeddev, median);
            situation = zmed > prm.thr_bb || zmed < -prm.thr_bb;
        }

        // Magnitude triggers (:214-241) into trig_all, or straight to the
        // flags (the stores only where some lane triggered).
        {
            const uint32_t mag_bits = situation ? ok_bits :
                    z_bits<EPL>(make_ztest(median, mediandev, prm.thr_mag),
                            [&](int j) { return (double)m[j]; }) & ok_bits;
            if (prm.window > 0)
            {
#pragma unroll
                for (int j = 0; j < EPL; ++j)
                    if (ch_ok[j]) trig_all[lane + 64 * j] = (mag_bits >> j) & 1u;
            }
            else if (__builtin_amdgcn_ballot_w64(mag_bits != 0))
            {
#pragma unroll
                for (int j = 0; j < EPL; ++j)
                    if ((mag_bits >> j) & 1u) set_flag(frow, j, P, lane);
            }
        }

        // Fluctuations (:245-339).
        if (t > 0)
        {
            double medianvar, mediandevvar;
            {
                auto kt = [&](int j) -> uint64_t {
                    return smp_ok[j] ? key_of(transit[j]) : ~(uint64_t)0;
                };
                medianvar = select_tracked<double, EPL, kCandRegs>(kt, k_s,
                        prm.ns, tk_var, (uint64_t*)cand, lane, 4);
            }
            {
                // MAD around the MAGNITUDE median (:292-295).
                auto kv = [&](int j) -> uint64_t {
                    return smp_ok[j] ? key_of(fabs(transit[j] - median)) :
                                       ~(uint64_t)0;
                };
                // |transit - median| sits about `median` above zero: move
                // its bracket with the magnitude median.
                if (tk_vdev.valid) tk_vdev.x += median - prev_median;
                mediandevvar = select_tracked<double, EPL, kCandRegs>(kv,
                        k_s, prm.ns, tk_vdev, (uint64_t*)cand, lane, 5);
            }
            const uint32_t var_bits = z_bits<EPL>(
                    make_ztest(medianvar, mediandevvar, prm.thr_var),
                    [&](int j) { return fabs(transit[j]); }) & ok_bits;
            if (prm.window > 0)
            {
#pragma unroll
                for (int j = 0; j < EPL; ++j)
                {
                    const int c = lane + 64 * j;
                    const uint32_t tv = (var_bits >> j) & 1u;
                    if (ch_ok[j]) trig_var[c] = tv;
                    if (tv) trig_all[c] = 1;
                }
            }
            else if (__builtin_amdgcn_ballot_w64(var_bits != 0))
            {
#pragma unroll
                for (int j = 0; j < EPL; ++j)
                {
                    if ((var_bits >> j) & 1u)
                    {
                        set_flag(frow, j, P, lane);
                        set_flag(fprev, j, P, lane);
                    }
                }
            }
        }

        // Window spread and flag stores: row t gets magnitude | variation
        // triggers, row t - 1 the variation triggers again (:311-338).
        if (prm.window > 0)
        {
            wave_sync();
#pragma unroll 1
            for (int j = 0; j < EPL; ++j)
            {
                const int c = lane + 64 * j;
                if (!ch_ok[j]) continue;
                if (spread(trig_all, c, C, prm.window))
                    set_flag(frow, j, P, lane);
                if (t > 0 && spread(trig_var, c, C, prm.window))
                    set_flag(fprev, j, P, lane);
            }
            wave_sync();
        }
#pragma unroll
        for (int j = 0; j < EPL; ++j) prev[j] = m[j];
        prev_median = median;
        hpos = hpos + 1 == prm.wmh ? 0 : hpos + 1;
    }
}

template<typename FP, int EPL, bool FULL>
sdp_Error launch_epl(const FP* vis, int32_t* flags, const FlagParams& prm)
{
    sdp_Error st = SDP_SUCCESS;
    const int64_t streams = prm.B * prm.P;
    const unsigned blocks = (unsigned)((streams + kWaves - 1) / kWaves);
    const size_t lds = kWaves * lds_per_wave(prm.wmh, prm.C);
    auto run = [&](auto kern) {
        if (lds > 64 * 1024)
            SDP_HIP_CHECK(hipFuncSetAttribute((const void*)kern,
                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds),
                    &st);
        kern<<<blocks, 64 * kWaves, lds, 0>>>(vis, flags, prm);
    };
    if (prm.wmh <= 64)
        run(k_flagger<FP, EPL, 1, FULL>);
    else
        run(k_flagger<FP, EPL, 16, FULL>);
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<typename FP, int EPL>
sdp_Error launch_full(const FP* vis, int32_t* flags, const FlagParams& prm)
{
    if (prm.step == 1 && prm.C == 64 * EPL)
        return launch_epl<FP, EPL, true>(vis, flags, prm);
    return launch_epl<FP, EPL, false>(vis, flags, prm);
}

template<typename FP>
sdp_Error launch(const FP* vis, int32_t* flags, const FlagParams& prm)
{
    const int epl = (prm.C + 63) / 64;
    if (epl <= 1) return launch_full<FP, 1>(vis, flags, prm);
    if (epl <= 2) return launch_full<FP, 2>(vis, flags, prm);
    if (epl <= 4) return launch_full<FP, 4>(vis, flags, prm);
    if (epl <= 8) return launch_full<FP, 8>(vis, flags, prm);
    if (epl <= 16) return launch_full<FP, 16>(vis, flags, prm);
    return launch_full<FP, 32>(vis, flags, prm);
}

// Argument checks of the reference (check_params_dynamic,
// sdp_flagger.cpp:10-57), same codes and messages, plus the shape and
// size limits of this implementation.
void check_params(const sdp_Mem* vis, sdp_Mem* flags, sdp_Error* status)
{
    if (*status) return;
    if (sdp_mem_is_read_only(flags))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Output flags must be writable.");
        return;
    }
    if (!sdp_mem_is_c_contiguous(vis) || !sdp_mem_is_c_contiguous(flags))
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("All arrays must be C contiguous.");
        return;
    }
    if (sdp_mem_num_dims(vis) != 4 || sdp_mem_num_dims(flags) != 4)
    {
        *status = SDP_ERR_RUNTIME;
        SDP_LOG_ERROR("Visibility and flags arrays must be 4D.");
        return;
    }
    if (!sdp_mem_is_complex(vis))
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Visibilities must be complex.");
        return;
    }
    if (sdp_mem_type(flags) != SDP_MEM_INT)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Flags must be integers.");
        return;
    }
    if (sdp_mem_location(vis) != sdp_mem_location(flags))
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("All arrays must be in the same memory location.");
        return;
    }
    for (int d = 0; d < 4; ++d)
    {
        if (sdp_mem_shape_dim(vis, d) != sdp_mem_shape_dim(flags, d))
        {
            *status = SDP_ERR_INVALID_ARGUMENT;
            SDP_LOG_ERROR("Flags must have the shape of the visibilities.");
            return;
        }
    }
}

} // namespace

extern "C" {

void sdp_flagger_dynamic_threshold(
        const sdp_Mem* vis,
        sdp_Mem* flags,
        const double alpha,
        const double threshold_magnitudes,
        const double threshold_variations,
        const double threshold_broadband,
        const int sampling_step,
        const int window,
        const int window_median_history,
        sdp_Error* status)
{
    check_params(vis, flags, status);
    if (*status) return;
    const sdp_MemType vt = sdp_mem_type(vis);
    if (vt != SDP_MEM_COMPLEX_FLOAT && vt != SDP_MEM_COMPLEX_DOUBLE)
    {
        *status = SDP_ERR_DATA_TYPE;
        SDP_LOG_ERROR("Unsupported data type(s): visibilities and "
                "thresholds arrays must have the same precision.");
        return;
    }
    FlagParams prm;
    prm.T = sdp_mem_shape_dim(vis, 0);
    prm.B = sdp_mem_shape_dim(vis, 1);
    prm.C = (int)sdp_mem_shape_dim(vis, 2);
    prm.P = (int)sdp_mem_shape_dim(vis, 3);
    prm.step = sampling_step;
    prm.window = window < 0 ? 0 : window;
    prm.wmh = window_median_history;
    prm.alpha = alpha;
    prm.thr_mag = threshold_magnitudes;
    prm.thr_var = threshold_variations;
    prm.thr_bb = threshold_broadband;
    if (prm.C < 1 || prm.C > kMaxChannels || sampling_step < 1 ||
            sampling_step > prm.C || prm.wmh < 1 || prm.wmh > kMaxHistory)
    {
        *status = SDP_ERR_INVALID_ARGUMENT;
        SDP_LOG_ERROR("Flagger limits: 1 <= num_channels <= %d, "
                "1 <= sampling_step <= num_channels, "
                "1 <= window_median_history <= %d", kMaxChannels, kMaxHistory);
        return;
    }
    prm.ns = prm.C / sampling_step;
    const int64_t n = sdp_mem_num_elements(vis);
    if (n == 0 || prm.P == 0) return;
    if (!sdp_hip::device_available())
    {
        *status = SDP_ERR_MEM_LOCATION;
        SDP_LOG_ERROR("No GPU available for the flagger.");
        return;
    }
    const size_t vbytes = (size_t)n * sdp_mem_type_size(vt);
    const size_t fbytes = (size_t)n * sizeof(int32_t);
    const bool on_host = sdp_mem_location(vis) == SDP_MEM_CPU;
    const void* d_vis = sdp_mem_data_const(vis);
    void* d_flags = sdp_mem_data(flags);
    void* tmp_vis = nullptr;
    void* tmp_flags = nullptr;
    if (on_host)
    {
        // Host arrays are staged through device memory; the flagger itself
        // runs on the GPU (there is no CPU path).
        SDP_HIP_CHECK(hipMalloc(&tmp_vis, vbytes), status);
        SDP_HIP_CHECK(hipMalloc(&tmp_flags, fbytes), status);
        if (*status)
        {
            (void)hipFree(tmp_vis);
            (void)hipFree(tmp_flags);
            *status = SDP_ERR_MEM_ALLOC_FAILURE;
            return;
        }
        SDP_HIP_CHECK(hipMemcpy(tmp_vis, d_vis, vbytes,
                hipMemcpyHostToDevice), status);
        SDP_HIP_CHECK(hipMemcpy(tmp_flags, d_flags, fbytes,
                hipMemcpyHostToDevice), status);
        d_vis = tmp_vis;
    }
    int32_t* f = (int32_t*)(on_host ? tmp_flags : d_flags);
    if (!*status)
    {
        const sdp_Error e = (vt == SDP_MEM_COMPLEX_FLOAT) ?
                launch<float>((const float*)d_vis, f, prm) :
                launch<double>((const double*)d_vis, f, prm);
        if (e) *status = e;
#ifdef SDP_FLAGGER_STATS
        unsigned long long st[6][7];
        (void)hipDeviceSynchronize();
        (void)hipMemcpyFromSymbol(st, HIP_SYMBOL(g_flag_stats), sizeof(st));
        for (int i = 0; i < 6; ++i)
            fprintf(stderr, "flagger stat %d: init %llu hit_cand %llu "
                    "hit_all %llu miss %llu probes_cand %llu probes_all %llu "
                    "hit_second %llu\n", i, st[i][0], st[i][1], st[i][2],
                    st[i][3], st[i][4], st[i][5], st[i][6]);
        memset(st, 0, sizeof(st));
        (void)hipMemcpyToSymbol(HIP_SYMBOL(g_flag_stats), st, sizeof(st));
#endif
    }
    if (on_host)
    {
        if (!*status)
            SDP_HIP_CHECK(hipMemcpy(d_flags, tmp_flags, fbytes,
                    hipMemcpyDeviceToHost), status);
        (void)hipFree(tmp_vis);
        (void)hipFree(tmp_flags);
    }
}

} // extern "C"
