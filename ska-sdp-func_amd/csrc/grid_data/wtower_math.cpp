// Host-side kernel math of the w-towers gridder. See wtower_math.h.
#include <algorithm>
#include <cmath>

#include "wtower_math.h"

namespace sdp_wt {

namespace {

constexpr double kPi = 3.14159265358979323846;

// Symmetric tridiagonal matrix (diag d, off-diagonal e[k] between k, k+1)
// of the prolate operator in the orthonormal basis sqrt((2r+1)/2) P_r,
// r = 0, 2, 4, ... (m = 0, even functions).
void prolate_matrix(double c, int n, std::vector<double>& d,
        std::vector<double>& e)
{
    const double c2 = c * c;
    d.assign(n, 0.0);
    e.assign(n, 0.0);
    for (int k = 0; k < n; ++k)
    {
        const double r = 2.0 * k;
        d[k] = r * (r + 1) + c2 * (2 * r * (r + 1) - 1) /
                ((2 * r - 1) * (2 * r + 3));
        e[k] = c2 * (r + 1) * (r + 2) /
                ((2 * r + 3) * std::sqrt((2 * r + 1) * (2 * r + 5)));
    }
}

// Number of eigenvalues below x (Sturm sequence count).
int sturm_count(const std::vector<double>& d, const std::vector<double>& e,
        double x)
{
    int count = 0;
    double q = 1.0;
    for (size_t k = 0; k < d.size(); ++k)
    {
        const double ek = (k == 0) ? 0.0 : e[k - 1];
        q = d[k] - x - (k == 0 ? 0.0 : ek * ek / q);
        if (q == 0.0) q = 1e-300;
        if (q < 0.0) ++count;
    }
    return count;
}

} // namespace

namespace {

// Lowest eigenpair of the symmetric tridiagonal (d, e): Sturm bisection for
// the eigenvalue, then inverse iteration; returns the unit eigenvector.
std::vector<double> lowest_eigenvector(const std::vector<double>& d,
        const std::vector<double>& e)
{
    const int n = (int)d.size();
    double lo = 1e300, hi = -1e300;
    for (int k = 0; k < n; ++k)
    {
        const double rad = std::fabs(k > 0 ? e[k - 1] : 0.0) + std::fabs(e[k]);
        lo = std::min(lo, d[k] - rad);
        hi = std::max(hi, d[k] + rad);
    }
    for (int it = 0; it < 200; ++it)
    {
        const double mid = 0.5 * (lo + hi);
        if (mid == lo || mid == hi) break;
        if (sturm_count(d, e, mid) >= 1) hi = mid; else lo = mid;
    }
    const double lambda = 0.5 * (lo + hi);
    std::vector<double> y(n, 1.0), b(n), cp(n), dp(n);
    const double shift = lambda - 1e-10 * std::max(1.0, std::fabs(lambda));
    for (int it = 0; it < 6; ++it)
    {
        b = y;
        double den = d[0] - shift;
        cp[0] = e[0] / den;
        dp[0] = b[0] / den;
        for (int k = 1; k < n; ++k)
        {
            den = (d[k] - shift) - e[k - 1] * cp[k - 1];
            cp[k] = (k < n - 1) ? e[k] / den : 0.0;
            dp[k] = (b[k] - e[k - 1] * dp[k - 1]) / den;
        }
        y[n - 1] = dp[n - 1];
        for (int k = n - 2; k >= 0; --k) y[k] = dp[k] - cp[k] * y[k + 1];
        double norm = 0.0;
        for (int k = 0; k < n; ++k) norm += y[k] * y[k];
        norm = std::sqrt(norm);
        for (int k = 0; k < n; ++k) y[k] /= norm;
    }
    return y;
}

} // namespace

Pswf make_pswf_order(double c, int m)
{
    if (m <= 0) return make_pswf(c);
    // Prolate operator -d/dx (1 - x^2) d/dx + m^2 / (1 - x^2) + c^2 x^2 in
    // the orthonormal basis of P_l^m, l = m, m + 2, ...: diagonal
    // l (l + 1) + c^2 <x^2>_ll, off-diagonal c^2 a_l a_{l+1}, with
    // x P_l^m = a_l P_{l+1}^m + a_{l-1} P_{l-1}^m (normalised),
    // a_j = sqrt(((j + 1)^2 - m^2) / ((2j + 1)(2j + 3))).
    const int n = std::max(40, (int)(c) + 40);
    auto a = [m](double j) {
        return std::sqrt(std::max(0.0, ((j + 1) * (j + 1) - (double)m * m) /
                ((2 * j + 1) * (2 * j + 3))));
    };
    std::vector<double> d(n), e(n);
    const double c2 = c * c;
    for (int k = 0; k < n; ++k)
    {
        const double l = m + 2.0 * k;
        const double am = (l - 1 >= m) ? a(l - 1) : 0.0;
        d[k] = l * (l + 1) + c2 * (a(l) * a(l) + am * am);
        e[k] = c2 * a(l) * a(l + 1);
    }
    const std::vector<double> y = lowest_eigenvector(d, e);
    Pswf p;
    p.c = c;
    p.m = m;
    p.coef.resize(n);
    for (int k = 0; k < n; ++k)
    {
        const double l = m + 2.0 * k;
        // normalised -> plain P_l^m: sqrt((2l + 1) / 2 (l - m)! / (l + m)!)
        p.coef[k] = y[k] * std::sqrt((2 * l + 1) / 2.0 *
                std::exp(std::lgamma(l - m + 1) - std::lgamma(l + m + 1)));
    }
    double target = 1.0;
    for (int j = 1; j <= m; ++j) target *= (2.0 * j - 1.0);
    const double at0 = p(0.0);
    for (int k = 0; k < n; ++k) p.coef[k] *= target / at0;
    return p;
}

Pswf make_pswf(double c)
{
    Pswf p;
    p.c = c;
    const int n = std::max(40, (int)(c) + 40);
    std::vector<double> d, e;
    prolate_matrix(c, n, d, e);
    // Lowest eigenvalue: bisection on the Sturm count (Gershgorin bounds).
    double lo = 1e300, hi = -1e300;
    for (int k = 0; k < n; ++k)
    {
        const double rad = std::fabs(k > 0 ? e[k - 1] : 0.0) + std::fabs(e[k]);
        lo = std::min(lo, d[k] - rad);
        hi = std::max(hi, d[k] + rad);
    }
    for (int it = 0; it < 200; ++it)
    {
        const double mid = 0.5 * (lo + hi);
        if (mid == lo || mid == hi) break;
        if (sturm_count(d, e, mid) >= 1) hi = mid; else lo = mid;
    }
    const double lambda = 0.5 * (lo + hi);
    // Eigenvector: inverse iteration with a tridiagonal (Thomas) solve.
    std::vector<double> y(n, 1.0), b(n), cp(n), dp(n);
    const double shift = lambda - 1e-10 * std::max(1.0, std::fabs(lambda));
    for (int it = 0; it < 6; ++it)
    {
        b = y;
        // Solve (T - shift I) y = b.
        double den = d[0] - shift;
        cp[0] = e[0] / den;
        dp[0] = b[0] / den;
        for (int k = 1; k < n; ++k)
        {
            den = (d[k] - shift) - e[k - 1] * cp[k - 1];
            cp[k] = (k < n - 1) ? e[k] / den : 0.0;
            dp[k] = (b[k] - e[k - 1] * dp[k - 1]) / den;
        }
        y[n - 1] = dp[n - 1];
        for (int k = n - 2; k >= 0; --k) y[k] = dp[k] - cp[k] * y[k + 1];
        double norm = 0.0;
        for (int k = 0; k < n; ++k) norm += y[k] * y[k];
        norm = std::sqrt(norm);
        for (int k = 0; k < n; ++k) y[k] /= norm;
    }
    // Coefficients of the unnormalised Legendre polynomials P_2k.
    p.coef.resize(n);
    for (int k = 0; k < n; ++k)
        p.coef[k] = y[k] * std::sqrt((4.0 * k + 1) / 2.0);
    const double at0 = p(0.0);
    for (int k = 0; k < n; ++k) p.coef[k] /= at0;
    return p;
}

double Pswf::operator()(double x) const
{
    if (m > 0)
    {
        // Sum of coef[k] P_{m+2k}^m(x): P_m^m = (2m - 1)!! (1 - x^2)^(m/2),
        // P_{m+1}^m = (2m + 1) x P_m^m,
        // (l - m + 1) P_{l+1}^m = (2l + 1) x P_l^m - (l + m) P_{l-1}^m.
        double pmm = std::pow(std::max(0.0, 1.0 - x * x), 0.5 * m);
        for (int j = 1; j <= m; ++j) pmm *= (2.0 * j - 1.0);
        double p_prev = pmm, p_cur = (2.0 * m + 1) * x * pmm;
        double sum = coef.empty() ? 0.0 : coef[0] * pmm;
        const int lmax = m + 2 * ((int)coef.size() - 1);
        for (int l = m + 1; l < lmax; ++l)
        {
            const double p_next = ((2.0 * l + 1) * x * p_cur -
                    (l + m) * p_prev) / (l - m + 1);
            p_prev = p_cur;
            p_cur = p_next;
            if ((l + 1 - m) % 2 == 0) sum += coef[(l + 1 - m) / 2] * p_cur;
        }
        return sum;
    }
    // Sum of coef[k] P_2k(x), Legendre recurrence up to degree 2 (n - 1).
    double p_prev = 1.0, p_cur = x, sum = coef.empty() ? 0.0 : coef[0];
    const int nmax = 2 * ((int)coef.size() - 1);
    for (int deg = 1; deg < nmax; ++deg)
    {
        const double p_next = ((2.0 * deg + 1) * x * p_cur - deg * p_prev) /
                (deg + 1);
        p_prev = p_cur;
        p_cur = p_next;
        if ((deg + 1) % 2 == 0) sum += coef[(deg + 1) / 2] * p_cur;
    }
    return sum;
}

std::vector<double> generate_pswf(double c, int size, bool end_correction)
{
    const Pswf p = make_pswf(c);
    std::vector<double> out(size, 0.0);
    out[size / 2] = p(0.0);
    for (int i = 1; i < size / 2; ++i)
    {
        const double v = p(2.0 * i / size);
        out[size / 2 + i] = v;
        out[size / 2 - i] = v;
    }
    if (end_correction && size % 2 == 0) out[0] = 1e-15;
    return out;
}

std::vector<double> make_kernel(const std::vector<double>& window,
        int oversampling)
{
    const int support = (int)window.size();
    const double inv_support = 1.0 / support;
    const double inv_os = 1.0 / oversampling;
    const int half = support / 2;
    std::vector<double> kernel((size_t)(oversampling + 1) * support);
    for (int i = 0; i <= oversampling; ++i)
    {
        for (int s_out = 0; s_out < support; ++s_out)
        {
            const double du = (double)(i - oversampling);
            const double u = (s_out - half) - du * inv_os;
            double val = 0.0;
            for (int s_in = 0; s_in < support; ++s_in)
            {
                const double l = (s_in - half) * inv_support;
                val += window[s_in] * std::cos(2 * kPi * u * l);
            }
            kernel[(size_t)i * support + s_out] = val * inv_support;
        }
    }
    return kernel;
}

std::vector<double> make_pswf_kernel(int support, int oversampling)
{
    std::vector<double> pswf = generate_pswf(support * (kPi / 2), support,
            false);
    if (support % 2 == 0) pswf[0] = 1e-15;
    return make_kernel(pswf, oversampling);
}

std::vector<std::complex<double> > make_w_pattern(int subgrid_size,
        double theta, double shear_u, double shear_v, double w_step)
{
    const int half = subgrid_size / 2;
    std::vector<std::complex<double> > w((size_t)subgrid_size * subgrid_size);
    for (int il = 0; il < subgrid_size; ++il)
    {
        for (int im = 0; im < subgrid_size; ++im)
        {
            const double l = (il - half) * theta / subgrid_size;
            const double m = (im - half) * theta / subgrid_size;
            const double n = lm_to_n(l, m, shear_u, shear_v);
            const double phase = 2.0 * kPi * w_step * n;
            w[(size_t)il * subgrid_size + im] =
                    std::complex<double>(std::cos(phase), std::sin(phase));
        }
    }
    return w;
}

double determine_w_step(double theta, double fov, double shear_u,
        double shear_v, double x0)
{
    if (x0 == 0.0) x0 = fov / theta;
    const double v1 = lm_to_n(-fov / 2.0, -fov / 2.0, shear_u, shear_v);
    const double v2 = lm_to_n(fov / 2.0, -fov / 2.0, shear_u, shear_v);
    const double v3 = lm_to_n(-fov / 2.0, fov / 2.0, shear_u, shear_v);
    const double v4 = lm_to_n(fov / 2.0, fov / 2.0, shear_u, shear_v);
    const double fov_n = 2.0 * -std::min(std::min(v1, v2), std::min(v3, v4));
    const double theta_n = fov_n / x0;
    return 1.0 / theta_n;
}

} // namespace sdp_wt
