// MI355X-native dynamic-threshold RFI flagger.
//
// Replaces src/ska-sdp-func/visibility/sdp_flagger.cpp (ska-sdp-func 1.2.2)
// with bit-identical results. The reference walks every (baseline, pol)
// stream sequentially in time with 3-4 qsorts of <= num_channels doubles
// per step (:125-339). Here one 64-lane wave owns a stream: the channels of
// a time step live in registers (channel c in lane c % 64, slot c / 64),
// and every median is an exact order statistic found by a bitwise binary
// search over the IEEE bit patterns (all the values ranked are >= 0, so
// bit-pattern order is value order) with one ballot + scalar popcount per
// register per bit: no sort, no LDS traffic, no barriers. The stream state
// (previous magnitudes, transit scores) stays in registers across time
// steps; the median history is a per-wave LDS ring; window flagging reads
// trigger bytes from LDS. Flags are written only where set (idempotent
// stores of 1), so the output keeps whatever the caller's array held.
#include <cmath>
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

// k-th smallest (0-based) of the values v[j] with ok[j], over the wave.
// Bitwise binary search on the bit patterns of non-negative doubles:
// prefix ends as the largest key with #(key < prefix) <= k, which is the
// k-th order statistic itself. Bits below low_bit are known to be zero in
// every candidate (f32-derived magnitudes: 29) and are skipped.
template<int N>
__device__ __forceinline__ double select_kth(const double (&v)[N],
        const bool (&ok)[N], int k, int low_bit)
{
    uint64_t key[N];
#pragma unroll
    for (int j = 0; j < N; ++j) key[j] = (uint64_t)__double_as_longlong(v[j]);
    uint64_t prefix = 0;
    for (int bit = 62; bit >= low_bit; --bit)
    {
        const uint64_t cand = prefix | (1ull << bit);
        int cnt = 0;
#pragma unroll
        for (int j = 0; j < N; ++j)
            cnt += __popcll(__ballot(ok[j] && key[j] < cand));
        if (cnt <= k) prefix = cand;
    }
    return __longlong_as_double((long long)prefix);
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

__device__ __forceinline__ void wave_sync()
{
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_wave_barrier();
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

template<typename FP, int EPL, int HEPL>
__global__ __launch_bounds__(64 * kWaves) void k_flagger(
        const FP* __restrict__ vis, int32_t* __restrict__ flags,
        FlagParams prm)
{
#pragma clang fp contract(off)
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    const int64_t stream = (int64_t)blockIdx.x * kWaves + wave;
    if (stream >= prm.B * prm.P) return;   // whole wave
    const int64_t b = stream / prm.P;
    const int p = (int)(stream % prm.P);
    const int C = prm.C, P = prm.P;
    // Per-wave LDS: median history ring | trigger bytes (all, variation).
    const size_t per_wave = (size_t)prm.wmh * 8 + 2 * (size_t)((C + 15) & ~15);
    unsigned char* base = smem + per_wave * wave;
    double* hist = (double*)base;
    uint8_t* trig_all = base + (size_t)prm.wmh * 8;
    uint8_t* trig_var = trig_all + ((C + 15) & ~15);
    const int low_bit_mag = sizeof(FP) == 4 ? 29 : 0;
    const int k_s = mid_index(prm.ns);

    bool ch_ok[EPL], smp_ok[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j)
    {
        const int c = lane + 64 * j;
        ch_ok[j] = c < C;
        smp_ok[j] = c < C && (c % prm.step) == 0 && (c / prm.step) < prm.ns;
    }
    double prev[EPL], transit[EPL];
#pragma unroll
    for (int j = 0; j < EPL; ++j) prev[j] = transit[j] = 0.0;

    const int64_t time_block = prm.B * (int64_t)C * P;
    for (int64_t t = 0; t < prm.T; ++t)
    {
        const int64_t row = t * time_block + b * (int64_t)C * P + p;
        double m[EPL];
#pragma unroll
        for (int j = 0; j < EPL; ++j)
        {
            m[j] = 0.0;
            if (ch_ok[j])
            {
                const FP* z = vis + 2 * (row + (int64_t)(lane + 64 * j) * P);
                m[j] = mag_of(z[0], z[1]);
            }
        }
        // Magnitude median and MAD over the sampled channels (:170-178).
        const double median = select_kth<EPL>(m, smp_ok, k_s, low_bit_mag);
        double dv[EPL];
#pragma unroll
        for (int j = 0; j < EPL; ++j) dv[j] = fabs(m[j] - median);
        const double mediandev = select_kth<EPL>(dv, smp_ok, k_s, 0);

        // Broadband: median history of the last min(t + 1, wmh) steps.
        if (lane == 0) hist[t % prm.wmh] = median;
        wave_sync();
        const int medwindow = (int)((t + 1 < prm.wmh) ? t + 1 : prm.wmh);
        bool situation = false;
        if (t != 0)
        {
            double hv[HEPL];
            bool hok[HEPL];
#pragma unroll
            for (int j = 0; j < HEPL; ++j)
            {
                const int tt = lane + 64 * j;
                hok[j] = tt < medwindow;
                hv[j] = hok[j] ? hist[(t - tt) % prm.wmh] : 0.0;
            }
            const int k_h = mid_index(medwindow);
            const double medmed = select_kth<HEPL>(hv, hok, k_h, 0);
#pragma unroll
            for (int j = 0; j < HEPL; ++j) hv[j] = fabs(hv[j] - medmed);
            const double medmeddev = select_kth<HEPL>(hv, hok, k_h, 0);
            const double zmed = modified_zscore(medmed, medmeddev, median);
            situation = zmed > prm.thr_bb || zmed < -prm.thr_bb;
        }

        // Magnitude triggers (:214-241).
        bool trig[EPL], tv[EPL];
#pragma unroll
        for (int j = 0; j < EPL; ++j)
        {
            const double z = modified_zscore(median, mediandev, m[j]);
            trig[j] = ch_ok[j] &&
                    (z > prm.thr_mag || z < -prm.thr_mag || situation);
            tv[j] = false;
        }

        // Fluctuations (:245-339).
        if (t > 0)
        {
#pragma unroll
            for (int j = 0; j < EPL; ++j)
            {
                const double rate = fabs(prev[j] - m[j]);
                transit[j] = (t == 1) ? rate :
                        prm.alpha * rate + (1 - prm.alpha) * transit[j];
            }
            const double medianvar = select_kth<EPL>(transit, smp_ok, k_s, 0);
            // MAD around the MAGNITUDE median (:292-295).
#pragma unroll
            for (int j = 0; j < EPL; ++j) dv[j] = fabs(transit[j] - median);
            const double mediandevvar = select_kth<EPL>(dv, smp_ok, k_s, 0);
#pragma unroll
            for (int j = 0; j < EPL; ++j)
            {
                const double z = modified_zscore(medianvar, mediandevvar,
                        fabs(transit[j]));
                tv[j] = ch_ok[j] && (z > prm.thr_var || z < -prm.thr_var);
            }
        }

        // Window spread and flag stores: row t gets magnitude | variation
        // triggers, row t - 1 the variation triggers again (:311-338).
#pragma unroll
        for (int j = 0; j < EPL; ++j)
        {
            const int c = lane + 64 * j;
            if (c < C)
            {
                trig_all[c] = (trig[j] || tv[j]) ? 1 : 0;
                trig_var[c] = tv[j] ? 1 : 0;
            }
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < EPL; ++j)
        {
            const int c = lane + 64 * j;
            if (c >= C) continue;
            if (spread(trig_all, c, C, prm.window))
                flags[row + (int64_t)c * P] = 1;
            if (t > 0 && spread(trig_var, c, C, prm.window))
                flags[row - time_block + (int64_t)c * P] = 1;
        }
        wave_sync();
#pragma unroll
        for (int j = 0; j < EPL; ++j) prev[j] = m[j];
    }
}

template<typename FP, int EPL>
sdp_Error launch_epl(const FP* vis, int32_t* flags, const FlagParams& prm)
{
    sdp_Error st = SDP_SUCCESS;
    const int64_t streams = prm.B * prm.P;
    const unsigned blocks = (unsigned)((streams + kWaves - 1) / kWaves);
    const size_t lds = kWaves * ((size_t)prm.wmh * 8 +
            2 * (size_t)((prm.C + 15) & ~15));
    if (prm.wmh <= 64)
    {
        if (lds > 64 * 1024)
            SDP_HIP_CHECK(hipFuncSetAttribute(
                    (const void*)k_flagger<FP, EPL, 1>,
                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), &st);
        k_flagger<FP, EPL, 1><<<blocks, 64 * kWaves, lds, 0>>>(vis, flags,
                prm);
    }
    else
    {
        if (lds > 64 * 1024)
            SDP_HIP_CHECK(hipFuncSetAttribute(
                    (const void*)k_flagger<FP, EPL, 16>,
                    hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds), &st);
        k_flagger<FP, EPL, 16><<<blocks, 64 * kWaves, lds, 0>>>(vis, flags,
                prm);
    }
    SDP_HIP_CHECK_LAUNCH(&st);
    return st;
}

template<typename FP>
sdp_Error launch(const FP* vis, int32_t* flags, const FlagParams& prm)
{
    const int epl = (prm.C + 63) / 64;
    if (epl <= 1) return launch_epl<FP, 1>(vis, flags, prm);
    if (epl <= 2) return launch_epl<FP, 2>(vis, flags, prm);
    if (epl <= 4) return launch_epl<FP, 4>(vis, flags, prm);
    if (epl <= 8) return launch_epl<FP, 8>(vis, flags, prm);
    if (epl <= 16) return launch_epl<FP, 16>(vis, flags, prm);
    return launch_epl<FP, 32>(vis, flags, prm);
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
