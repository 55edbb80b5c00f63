/* MI355X-native FFT wrapper: drop-in C ABI on rocFFT.
 *
 * Replaces src/ska-sdp-func/fourier_transforms/sdp_fft.h:28-128 of
 * ska-sdp-func 1.2.2 (impl sdp_fft.cpp:295-1191, cuFFT plan :362-448,
 * kernels sdp_fft.cu:11-29; bound from Python by
 * src/ska_sdp_func/fourier_transforms/fft.py:13-92).
 *
 * Complex-to-complex, unnormalised both ways (inverse = +i exponent), 1-,
 * 2- or 3-D, batched over the first dimension when the arrays have one
 * more dimension than the transform. The transform always runs on the GPU:
 * host (CPU) arrays are staged through device memory.
 */
#ifndef SKA_SDP_PROC_FUNC_FFT_H_
#define SKA_SDP_PROC_FUNC_FFT_H_

#include "ska-sdp-func/utility/sdp_mem.h"

#ifdef __cplusplus
extern "C" {
#endif

struct sdp_Fft;
typedef struct sdp_Fft sdp_Fft;

/* Plan for the given arrays (same location, type and shape; C-contiguous;
 * complex float or complex double), reference .h:60-66. */
sdp_Fft* sdp_fft_create(
        const sdp_Mem* input,
        const sdp_Mem* output,
        int32_t num_dims_fft,
        int32_t is_forward,
        sdp_Error* status
);

/* Transform input into output (may be the same array); the arrays must
 * match those of the plan, .h:76-81. */
void sdp_fft_exec(
        sdp_Fft* fft,
        sdp_Mem* input,
        sdp_Mem* output,
        sdp_Error* status
);

/* phase, FFT in place, phase, and 1 / N if norm, .h:94-99. */
void sdp_fft_exec_shift(
        sdp_Fft* fft,
        sdp_Mem* data,
        int norm,
        sdp_Error* status
);

/* .h:106. */
void sdp_fft_free(sdp_Fft* fft);

/* data *= 1 / (dim0 * dim1) for a 2-D complex array, .h:116. */
void sdp_fft_norm(sdp_Mem* data, sdp_Error* status);

/* data *= (-1)^(i + j) (fftshift by checkerboard) for a 1-D or 2-D
 * complex array, .h:128. */
void sdp_fft_phase(sdp_Mem* data, sdp_Error* status);

/* ---- MI355X extension (not in the reference ABI) ----------------------
 * The w-stack plane transform of the w-towers gridder: a G x G complex-float
 * GPU array, G a power of two in [1024, 16384], transformed in place
 * (unnormalised; forward e^-, inverse e^+) by the fused three-pass FFT.
 * The output's row k is STORED at row N1 (k mod N2) + k / N2 (G = N1 N2,
 * N2 = sdp_fft_permuted_n2(G)); columns are in natural order. */
void sdp_fft_2d_inplace_permuted(sdp_Mem* data, int is_forward,
        sdp_Error* status);
int sdp_fft_permuted_n2(int grid_size);

#ifdef __cplusplus
}
#endif

#endif
