// Fused image side of the w-stacking imager (sdp_grid_wstack_wtower.hip) on
// the FFT machinery of es_fft.hip: a w-stack plane's inverse FFT with the
// corrected image update in its last column pass (ref
// sdp_grid_wstack_wtower.cpp:686-711).
#ifndef SDP_ES_FFT_WSTACK_H_
#define SDP_ES_FFT_WSTACK_H_

#include "es_fft.h"
#include "wtower_plan.h"

namespace sdp_es {

// image (G x G, any AnyView kind) += grid_correct(checker(IFFT2(grid)) *
// norm) for a w-stack plane (cp: its correction, w_offset included); the
// grid buffer is used as scratch (in place). G a power of two in [1024,
// 16384] with tw its twiddles.
int fft2d_wstack_grid_image(float* grid, int grid_size, const FftTwiddles& tw,
        const sdp_wt::AnyView& image, float norm,
        const sdp_wt::CorrParams& cp, hipStream_t stream);

// grid = FFT2(checker(degrid_correct((float)image))) for a w-stack plane
// (cp: its correction, w_offset included), unnormalised forward transform
// with the stored-row permutation of fft2d_inplace_permuted; the prologue
// is read by the first column pass (no separate pass over the grid). G a
// power of two in [1024, 16384] with tw its twiddles.
int fft2d_wstack_image_to_grid(float* grid, int grid_size,
        const FftTwiddles& tw, const sdp_wt::AnyView& image,
        const sdp_wt::CorrParams& cp, hipStream_t stream);

// Sub-grid cut-out read by the first pass of subgrid_fft2d (degridding):
// element (a, b) of slot k's sub-grid is (-1)^(ou + ov) grid[row(gu)][gv]
// with gu = (ou + a) mod G, gv = (ov + b) mod G, (ou, ov) the origin of
// sub-grid task[k] (iu = min_iu + task / nv, iv = min_iv + task % nv, origin
// G / 2 - S / 2 + i * eff mod G), row() the plane FFT's stored-row
// permutation (perm_shift = log2 fft_perm_n2, or -1 for none). G even.
struct SubgridCut
{
    const float2* grid = nullptr;
    int G = 0;
    const int* task = nullptr;
    int nv = 1, min_iu = 0, min_iv = 0, eff = 0;
    int perm_shift = -1;
};

// Batched 2-D FFT of slots S x S complex-float sub-grids in place,
// unnormalised (forward e^-, inverse e^+, as rocFFT); tw: twiddles of size
// S. With cut (inverse only), the input is read from the plane grid
// instead of sub. S = 128 or 256.
bool subgrid_fft_supported(int subgrid_size);
int subgrid_fft2d(float* sub, int subgrid_size, int64_t slots, bool forward,
        const FftTwiddles& tw, const SubgridCut* cut, hipStream_t stream);

} // namespace sdp_es

#endif
