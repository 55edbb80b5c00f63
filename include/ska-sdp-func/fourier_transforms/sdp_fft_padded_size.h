/* Padded FFT size: drop-in C ABI.
 *
 * Replaces src/ska-sdp-func/fourier_transforms/sdp_fft_padded_size.h:25
 * of ska-sdp-func 1.2.2 (impl sdp_fft_padded_size.cpp:87-126).
 */
#ifndef SKA_SDP_FFT_PADDED_SIZE_H_
#define SKA_SDP_FFT_PADDED_SIZE_H_

#ifdef __cplusplus
extern "C" {
#endif

/* The smallest even number >= ceil(n * padding_factor) whose half has no
 * prime factor above 11. */
int sdp_fft_padded_size(int n, double padding_factor);

#ifdef __cplusplus
}
#endif

#endif
