// TEST INFRASTRUCTURE ONLY: runs the reference's ES parameter functions
// (sdp_gridder_uvw_es_fft_utils.cpp, linked from oracle/_ref) and prints
// their outputs as JSON lines.
//   params <N> <eps> <is_double>   -> grid_size, support, beta/support
//   tables <N> <G> <W> <beta>      -> quadrature + conv-corr tables
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <vector>

#include "ska-sdp-func/grid_data/sdp_gridder_uvw_es_fft_utils.h"

int main(int argc, char** argv)
{
    if (argc >= 5 && !strcmp(argv[1], "params"))
    {
        const int n = atoi(argv[2]);
        const double eps = atof(argv[3]);
        const int dbl = atoi(argv[4]);
        int g = 0, w = 0;
        double beta = 0.0;
        sdp_Error status = SDP_SUCCESS;
        sdp_calculate_params_from_epsilon(eps, n,
                dbl ? SDP_MEM_DOUBLE : SDP_MEM_FLOAT, g, w, beta, &status);
        printf("{\"N\": %d, \"eps\": %.17g, \"double\": %d, \"grid_size\": %d,"
                " \"support\": %d, \"beta\": %.17g, \"status\": %d}\n",
                n, eps, dbl, g, w, beta, (int)status);
        return 0;
    }
    if (argc >= 6 && !strcmp(argv[1], "tables"))
    {
        const int n = atoi(argv[2]), g = atoi(argv[3]), w = atoi(argv[4]);
        const double beta = atof(argv[5]);
        std::vector<double> qk(QUADRATURE_SUPPORT_BOUND, 0.0);
        std::vector<double> qn(QUADRATURE_SUPPORT_BOUND, 0.0);
        std::vector<double> qw(QUADRATURE_SUPPORT_BOUND, 0.0);
        std::vector<double> cc(n / 2 + 1, 0.0);
        sdp_generate_gauss_legendre_conv_kernel(n, g, w, beta, qk.data(),
                qn.data(), qw.data(), cc.data());
        auto dump = [](const char* name, const std::vector<double>& v) {
            printf("\"%s\": [", name);
            for (size_t i = 0; i < v.size(); ++i)
                printf("%s%.17g", i ? ", " : "", v[i]);
            printf("]");
        };
        printf("{\"N\": %d, \"G\": %d, \"W\": %d, \"beta\": %.17g, ", n, g, w,
                beta);
        dump("quad_kernel", qk); printf(", ");
        dump("quad_nodes", qn); printf(", ");
        dump("quad_weights", qw); printf(", ");
        dump("conv_corr", cc); printf("}\n");
        return 0;
    }
    fprintf(stderr, "usage: params N eps dbl | tables N G W beta\n");
    return 1;
}
