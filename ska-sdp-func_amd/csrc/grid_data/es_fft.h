// Pruned, fused 2-D FFT between the uv grid and the image crop (f32).
//
// Replaces, for power-of-two grids, the full G x G cuFFT/rocFFT transform
// plus the separate screen/correction kernels of the reference
// (sdp_gridder_uvw_es_fft.cpp:660-740 gridding, :781-890 degridding).
// Only the central M x M block of the transformed grid is ever used
// (M = 2 * (N / 2)), so the transform is done in three HBM passes, all in
// place in the grid buffer, with the image-plane work fused into the pass
// that touches the image:
//
//  gridding (inverse, +i):
//   rows   : length-G FFT of every grid row in LDS; keeps the M centre
//            outputs (row u of the buffer now holds H[u][0..M)).
//   col-A  : four-step, G = N1 * N2: length-N2 FFTs down the rows
//            u1 + N1 * n2 of each column, times W_G^(u1 k2), in place.
//   col-B  : length-N1 FFTs over the contiguous row block N1 * k2 + n1;
//            output row k = k2 + N2 * k1 of the centre goes straight into
//            the image with the screen + correction epilogue
//            (2-D: dirty = (dirty + checker * Re) / correction;
//             3-D: dirty += checker * Re(F * phasor(w)), per plane).
//  2-D gridding with 2048 <= G <= 8192 takes the real-output form instead
//   (es_fft.hip, k_rows_herm / k_cols_a_herm / k_cols_b_herm): the dirty
//   image keeps only Re of the transform, so the row pass transforms the
//   Hermitian part of the grid and packs each pair of row spectra into one
//   row of a half-length complex-to-real column transform; the column
//   passes move G/2 rows and the image row pairs 2m, 2m + 1 come from
//   Re / Im of one output row.
//  degridding (forward, -i): the mirror image -- the first column pass reads
//   the (corrected in place) image with the checker / phasor prologue, the
//   row pass zero-pads and writes every cell of the grid.
//
// HBM traffic per call at G = 8192, N = 5440: ~2.2 GB (rocFFT + separate
// screen: ~4.8 GB). Twiddles are read once per workgroup from a G-entry
// table computed in double on the host and kept in registers; in-register
// DFTs use compile-time roots of unity.
#ifndef SDP_ES_FFT_H_
#define SDP_ES_FFT_H_

#include <hip/hip_runtime.h>

#include "es_kernels.h"

namespace sdp_es {

// Grids the fused path handles: G a power of two in [1024, 16384].
bool fused_fft_supported(int grid_size);

// Twiddle table exp(-2 pi i m / G), m in [0, G), as float2 in device memory.
// Also owns the tile-occupancy table of the real-output gridding row pass
// (G / 64 tile rows of G / 1024 + 1 32-bit words, es_fft.hip).
struct FftTwiddles
{
    void* table = nullptr;
    void* masks = nullptr;
    int G = 0;
};
int fft_twiddles_create(int grid_size, FftTwiddles* tw);
void fft_twiddles_destroy(FftTwiddles* tw);

// Gridding, part 1: row pass + first column pass (in place on grid).
// tiles: nullptr (every cell of the grid is valid), or the bucketing's
// per-tile entry counts (BucketScratch::bin_count, block-major bins of
// 64 x 64 cells, ncoarse blocks per axis) when the scatter skipped the
// empty tiles: the row pass then reads nothing of those (they are zero).
int fft_grid_rows_cols(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, hipStream_t stream);
// The same in its two halves: the row pass alone, and column pass A of a
// grid whose row pass is done. Both passes are linear in the grid, so the
// row spectra of several grids (one per GPU) can be summed between them.
int fft_grid_rows(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, hipStream_t stream);
int fft_grid_cols_a(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, hipStream_t stream);
// Where the row pass leaves the data the column passes read: grid rows
// [0, rows), columns [col0, col0 + ncols) (real-output form: the G/2 + 1
// rows of the Hermitian part; complex form: every row).
void fft_grid_row_spectra(const ImageParams<float>& ip, int64_t* rows,
        int64_t* col0, int64_t* ncols);
// Gridding, part 2: last column pass + screen/correction into dirty.
int fft_grid_to_image(const ImageParams<float>& ip, int plane,
        const FftTwiddles& tw, float* grid, float* dirty, hipStream_t stream);

// Degridding: whether the two halves below run in the real-input form
// (half-length column transforms of the real image; 2-D, 2048 <= G <=
// 8192, the image corrected in place). Decided ONCE per call by the caller
// and passed to both halves, whose layouts must agree.
bool fft_degrid_real_form(const ImageParams<float>& ip,
        bool correct_in_place);
// Degridding, part 1: image prologue (2-D: correct dirty in place) + first
// column pass into the grid buffer.
int fft_image_cols(const ImageParams<float>& ip, int plane,
        const FftTwiddles& tw, float* dirty, bool correct_in_place,
        bool real_form, float* grid, hipStream_t stream);
// Degridding, part 2: second column pass + row pass writing the grid:
// every cell (tiles == nullptr), or only the tiles the gather of this
// bucketing reads (tiles = BucketScratch::bin_count of the degrid bins).
int fft_image_to_grid(const ImageParams<float>& ip, const FftTwiddles& tw,
        float* grid, const uint32_t* tiles, int ncoarse, bool real_form,
        hipStream_t stream);

// Whole-grid 2-D FFT of a complex-float G x G grid in place, unnormalised
// (forward e^-, inverse e^+, as rocFFT / cuFFT), in three passes (rows,
// then the four-step columns). The result's row k is stored at row
// fft_perm_row(k): callers read it through that permutation.
int fft2d_inplace_permuted(float* grid, int grid_size, bool forward,
        const FftTwiddles& tw, hipStream_t stream);
// N2 of the column split (G = N1 * N2; 0 if the size is not supported).
int fft_perm_n2(int grid_size);
// Storage row of the transform's row k: N1 * (k % N2) + k / N2.
__host__ __device__ __forceinline__ int64_t fft_perm_row(int64_t k,
        int64_t G, int n2)
{
    return n2 ? (G / n2) * (k % n2) + k / n2 : k;
}

} // namespace sdp_es

#endif
