/* TEST INFRASTRUCTURE ONLY -- CPU oracle for the dynamic-threshold RFI
 * flagger. Never linked into, or called by, the product library.
 *
 * A restatement of sdp_flagger_dynamic_threshold of ska-sdp-func 1.2.2,
 * src/ska-sdp-func/visibility/sdp_flagger.cpp:125-428, with the same
 * arithmetic in the same order and types:
 *   - |v| of std::complex<FP> is glibc cabsf / cabs, widened to double
 *     (samples are double arrays, :145-176);
 *   - "median" is sorted[round(0.5 n)] (:83-88), i.e. index (n + 1) / 2;
 *   - the MAD sorts |x - median| (:91-101); the variation MAD is taken
 *     around the MAGNITUDE median (:292-295);
 *   - modified z-score 0.6795 (x - med) / mad, mad == 0 -> 0 or 1e7
 *     (:104-122);
 *   - broadband test on the median history of the last
 *     min(t + 1, window_median_history) steps, ignored at t = 0 (:181-211);
 *   - window flagging uses c - w - 1 > 0, so channel 0 is never flagged as
 *     a neighbour (:224-240, :316-337);
 *   - the variation test also flags (t - 1) (:311-338);
 *   - EMA transit score alpha |d| + (1 - alpha) prev, reset at t == 1
 *     (:254-268);
 *   - sampling_step integer division drops tail channels (:145);
 *   - flags are only ever set to 1.
 * Differences, all outside the reference's defined behaviour: 64-bit
 * element positions (the reference's int positions overflow beyond 2^31
 * elements; its results there equal this oracle run per baseline chunk),
 * and n == 1 medians read sorted[0] instead of one past the end (only at
 * t == 0, where the reference discards the value).
 */
#include <complex.h>
/* glibc defines CMPLX / CMPLXF only for gcc >= 4.7; clang (the sanitizer
 * build, oracle/_cc.py) has the same builtin. */
#ifndef CMPLXF
#define CMPLXF(x, y) __builtin_complex((float)(x), (float)(y))
#endif
#ifndef CMPLX
#define CMPLX(x, y) __builtin_complex((double)(x), (double)(y))
#endif
#ifdef _OPENMP
#include <omp.h>
#endif
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

static int cmp_double(const void* a, const void* b)
{
    const double da = *(const double*)a, db = *(const double*)b;
    return (da > db) ? 1 : ((da < db) ? -1 : 0);
}

static int mid_index(int n)
{
    int m = (int)round(0.5 * n);
    return (m < n) ? m : n - 1;
}

/* arr sorted ascending */
static double median_calc(const double* arr, int n)
{
    return arr[mid_index(n)];
}

static double median_dev_calc(const double* arr, int n, double median,
        double* devs)
{
    for (int i = 0; i < n; ++i) devs[i] = fabs(arr[i] - median);
    qsort(devs, n, sizeof(double), cmp_double);
    return devs[mid_index(n)];
}

static double modified_zscore(double median, double mediandev, double val)
{
    if (mediandev == 0 && val == median) return 0;
    if (mediandev == 0 && val != median) return 10000000;
    return 0.6795 * (val - median) / mediandev;
}

static double mag_f32(const float* v, int64_t i)
{
    return (double)cabsf(CMPLXF(v[2 * i], v[2 * i + 1]));
}

static double mag_f64(const double* v, int64_t i)
{
    return cabs(CMPLX(v[2 * i], v[2 * i + 1]));
}

static void flag_window(int32_t* flags, int64_t row, int c, int window,
        int C, int P, int p)
{
    flags[row + (int64_t)c * P + p] = 1;
    for (int w = 0; w < window; ++w)
    {
        if (c - w - 1 > 0) flags[row + (int64_t)(c - w - 1) * P + p] = 1;
        if (c + w + 1 < C) flags[row + (int64_t)(c + w + 1) * P + p] = 1;
    }
}

static void flagger(const void* vis, int is_double, int32_t* flags,
        double alpha, double thr_mag, double thr_var, double thr_bb,
        int step, int window, int wmh, int64_t T, int64_t B, int C, int P)
{
    const int ns = C / step;
#pragma omp parallel
    {
        double* samples = calloc((size_t)(ns > 0 ? ns : 1), sizeof(double));
        double* devs = calloc((size_t)(C > wmh ? C : wmh) + 1, sizeof(double));
        double* transit = calloc((size_t)C, sizeof(double));
        double* transit_samples = calloc((size_t)(ns > 0 ? ns : 1),
                sizeof(double));
        double* history = calloc((size_t)T, sizeof(double));
        double* medarray = calloc((size_t)(wmh > 0 ? wmh : 1), sizeof(double));
#pragma omp for schedule(dynamic)
        for (int64_t b = 0; b < B; ++b)
        {
            for (int p = 0; p < P; ++p)
            {
                for (int64_t t = 0; t < T; ++t)
                {
                    const int64_t time_block = B * (int64_t)C * P;
                    const int64_t row = t * time_block + b * (int64_t)C * P;
                    const int64_t row_m1 = (t - 1) * time_block +
                            b * (int64_t)C * P;
                    int situation = 0;
                    const int medwindow = (int)((t + 1 < wmh) ? t + 1 : wmh);
#define MAG(pos) (is_double ? mag_f64((const double*)vis, (pos)) \
                            : mag_f32((const float*)vis, (pos)))
                    for (int s = 0; s < ns; ++s)
                        samples[s] = MAG(row + (int64_t)(s * step) * P + p);
                    qsort(samples, ns, sizeof(double), cmp_double);
                    const double median = median_calc(samples, ns);
                    const double mediandev = median_dev_calc(samples, ns,
                            median, devs);
                    history[t] = median;
                    for (int tt = 0; tt < medwindow; ++tt)
                        medarray[tt] = history[t - tt];
                    qsort(medarray, medwindow, sizeof(double), cmp_double);
                    const double medmed = median_calc(medarray, medwindow);
                    const double medmeddev = median_dev_calc(medarray,
                            medwindow, medmed, devs);
                    const double zmed = modified_zscore(medmed, medmeddev,
                            median);
                    if ((zmed > thr_bb || zmed < -thr_bb) && t != 0)
                        situation = 1;
                    for (int c = 0; c < C; ++c)
                    {
                        const double v1 = MAG(row + (int64_t)c * P + p);
                        const double z = modified_zscore(median, mediandev, v1);
                        if (z > thr_mag || z < -thr_mag || situation == 1)
                            flag_window(flags, row, c, window, C, P, p);
                    }
                    if (t > 0)
                    {
                        for (int c = 0; c < C; ++c)
                        {
                            const double v0 = MAG(row + (int64_t)c * P + p);
                            const double v1 = MAG(row_m1 + (int64_t)c * P + p);
                            const double rate = fabs(v1 - v0);
                            if (t == 1)
                                transit[c] = rate;
                            else
                                transit[c] = alpha * rate +
                                        (1 - alpha) * transit[c];
                        }
                        for (int s = 0; s < ns; ++s)
                            transit_samples[s] = fabs(transit[s * step]);
                        qsort(transit_samples, ns, sizeof(double), cmp_double);
                        const double medianvar = median_calc(transit_samples,
                                ns);
                        /* MAD around the magnitude median (:292-295). */
                        const double mediandevvar = median_dev_calc(
                                transit_samples, ns, median, devs);
                        for (int c = 0; c < C; ++c)
                        {
                            const double ts = fabs(transit[c]);
                            const double z = modified_zscore(medianvar,
                                    mediandevvar, ts);
                            if (z > thr_var || z < -thr_var)
                            {
                                flag_window(flags, row, c, window, C, P, p);
                                flag_window(flags, row_m1, c, window, C, P, p);
                            }
                        }
                    }
#undef MAG
                }
            }
        }
        free(samples);
        free(devs);
        free(transit);
        free(transit_samples);
        free(history);
        free(medarray);
    }
}

void oracle_flagger(const void* vis, int is_double, int32_t* flags,
        double alpha, double thr_mag, double thr_var, double thr_bb,
        int step, int window, int wmh, int64_t T, int64_t B, int C, int P)
{
    flagger(vis, is_double, flags, alpha, thr_mag, thr_var, thr_bb, step,
            window, wmh, T, B, C, P);
}

/* Threads of the OpenMP loop (the bench's CPU baseline sets the job's CPU
 * share); returns the count in effect. */
int oracle_flagger_set_threads(int n)
{
#ifdef _OPENMP
    if (n > 0) omp_set_num_threads(n);
    return omp_get_max_threads();
#else
    (void)n;
    return 1;
#endif
}

/* |v| as the reference computes it (glibc cabsf / cabs), for tests of the
 * device magnitude functions. */
void oracle_cabs_f32(const float* v, int64_t n, double* out)
{
    for (int64_t i = 0; i < n; ++i) out[i] = mag_f32(v, i);
}

void oracle_cabs_f64(const double* v, int64_t n, double* out)
{
    for (int64_t i = 0; i < n; ++i) out[i] = mag_f64(v, i);
}
