// HIP kernels of the MI355X-native ES-FFT (de)gridder: launch interface.
//
// Data path (one call; 3-D: one bucketing for every w-plane):
//   bucket_count -> scan_columns -> bucket_fill1 (+ scan_bins in its last
//   block) -> bucket_fill2 -> (grid) zero_shared_tiles + scatter_tab
//                             (degrid) gather_win
// Visibilities are bucketed by 64x64 grid tile (counting sort, LDS-private
// histograms per chunk of visibilities; records move in two levels: by
// super bin of S x S tiles with LDS-staged coalesced stores, then by tile).
// In grid mode a visibility is listed in every tile its support touches and
// each tile only accumulates the taps that fall inside it, so every grid
// cell has exactly one owning workgroup: the tile is accumulated in matrix-
// core accumulators and written to HBM ONCE with plain stores (no global
// atomics, no separate memset of the grid). Tiles with more entries than
// one work item takes are split into pieces that combine with global float
// atomics into a tile zeroed beforehand.
#ifndef SDP_ES_KERNELS_H_
#define SDP_ES_KERNELS_H_

#include <cstddef>
#include <cstdint>

#include <hip/hip_runtime.h>

namespace sdp_es {

constexpr int kTile = 64;              // grid tile edge (cells)
constexpr int kCoarse = 4;             // tiles per bin-numbering block edge
constexpr int kCoarseTile = kTile * kCoarse;   // 256 cells
constexpr int kBinsPerPass = 16384;    // LDS histogram capacity (64 KiB)
constexpr int kPiece = 4096;           // max entries per scatter work item
constexpr int kMaxChunks = 1024;       // chunks of visibilities per bucketing
constexpr int kCountChunks = 2;        // chunks per counting workgroup
                                       // (1: 62 / 47 us, 4: 67 / 46 us
                                       // against 54 / 41 at config 2)
constexpr int kGroupChunks = 16;       // chunks per level-2 group (and per
                                       // row of the tile count table;
                                       // 8 / 32: config-2 bucketing 0.277
                                       // -> 0.288 / 0.288 ms, round 6)
static_assert(kGroupChunks % kCountChunks == 0, "whole counting workgroups");
constexpr int kMaxSuperBins = 1024;    // super bins (first bucketing level)
constexpr int kMaxSuperTiles = 4096;   // tiles per super bin (S^2, S <= 64)
constexpr int kTapPolyPairs = 3;       // interior taps 1..6 of W = 8
constexpr int kTapPolyDeg = 8;         // fit ~1e-8, below f32 Horner (~9e-8 abs)

enum Mode { MODE_GRID = 0, MODE_DEGRID = 1 };

// Geometry + kernel coefficients of one pass, in working precision T.
template<typename T>
struct EsParams
{
    int G;              // grid side
    int support;        // W
    int do_w;           // w-stacking (3-D) path
    int plane;          // w-plane index processed (3-D), 0 in 2-D
    int ntiles;         // fine tiles per axis = ceil(G / kTile)
    int ncoarse;        // 4 x 4-tile blocks per axis = ceil(G / kCoarseTile)
    int ncbins;         // ncoarse^2
    int nbins;          // tile bins, block-major: 16 per 4 x 4-tile block
                        // (bin b: block b / 16, tile (b % 16) / 4, b % 4),
                        // so consecutive work items touch adjacent tiles
    int sshift;         // super bins (first bucketing level): S x S tiles,
    int nsuper;         // S = 1 << sshift >= 8, nsuper = ceil(ntiles / S)
    int nsbins;         // per axis, nsbins = nsuper^2 <= kMaxSuperBins
    int tstride;        // count table row: nbins tile counts | nsbins super
    T beta;             // full beta (table value * W)
    T uv_scale;         // G * pixel_size
    T w_scale;
    T min_plane_w;
    // f32 tile kernels at W = 8: interior taps d = 1..6 as polynomials of
    // s = 2 delta - 1 (delta = first tap - (pos - W / 2) in [0, 1)), pairs
    // (1, 2), (3, 4), (5, 6), coefficient k of both taps of a pair side by
    // side, (-1)^d folded in (es_tap_poly_fit).
    float tap_poly[kTapPolyPairs][kTapPolyDeg + 1][2];
    int tap_poly_ok;    // coefficients valid (f32 plan, W = 8)
};

// Chebyshev fit (double, nodes of degree kTapPolyDeg) of the interior ES
// taps of support 8 for the f32 beta, converted to monomials in s.
void es_tap_poly_fit(double beta_f32, float out[kTapPolyPairs]
        [kTapPolyDeg + 1][2]);

// Scratch owned by a plan (device pointers).
struct BucketScratch
{
    uint32_t* table = nullptr;      // [groups][nbins] tile counts / offsets
                                    // from the start, [chunks][nsbins]
                                    // super-bin counts / offsets at the end
                                    // (bucket_table_entries)
    uint32_t* bin_count = nullptr;  // [tstride]: tile then super-bin totals
    uint32_t* bin_start = nullptr;  // [nbins + 1]
    uint32_t* item_start = nullptr; // [nbins + 1]
    uint32_t* totals = nullptr;     // [2]: entries, items
    uint32_t* sb_start = nullptr;   // [nsbins + 1]: super-bin starts
    uint32_t* item_bin = nullptr;   // [item_capacity]: work item -> bin
    uint32_t item_capacity = 0;
    void* recs = nullptr;           // bucketed records (worst-case size)
    void* recs1 = nullptr;          // first level, by super bin (same size)
    size_t recs_bytes = 0;
    size_t table_entries = 0;
    bool gtable_dirty = true;       // group rows not known to be zero
};

// Number of visibility chunks used for a given visibility count and count
// table row length (the chunk-by-bin table stays below 2^31 bytes, the
// range of the buffer addressing in k_scan_columns).
int num_chunks(int64_t num_vis, int tstride);

// Entries of BucketScratch::table for nc chunks.
size_t bucket_table_entries(int nc, int nbins, int nsbins);

// Super-bin geometry for ntiles tiles per axis: sets sshift, nsuper, nsbins
// (the smallest S = 2^sshift >= 8 with ceil(ntiles / S)^2 <= kMaxSuperBins).
// Returns false if none exists within kMaxSuperTiles.
bool super_geometry(int ntiles, int* sshift, int* nsuper, int* nsbins);

// Bucketing, fully asynchronous: fills scratch.recs (sized by the caller
// for the worst case, 4 entries per visibility) and the work-item table;
// *n_items is the launch bound item_capacity (work items past the real
// count find kNoBin and exit), *n_entries is 0. 3-D (do_w): every
// visibility is bucketed ONCE for all w-planes (p.plane is ignored), with
// its plane coordinate pos_w in place of a w-tap; the tile kernels of
// plane p derive the tap (plane_tap) and skip the records off that plane.
// Record layouts:
//   grid, 2-D:  {pu, pv, vre*w, vim*w}
//   grid, 3-D:  {pu, pv, vre*w, vim*w*flip, pos_w, 0, 0, 0}
//   degrid:     {pu, pv, flip (2-D) | pos_w*flip (3-D), index bits}
template<typename T>
int bucket(const EsParams<T>& p, Mode mode, int64_t num_rows, int num_chan,
        const T* uvw, const T* freq, const T* vis, const T* weight,
        BucketScratch* s, hipStream_t stream, uint32_t* n_entries,
        uint32_t* n_items);

// Grid-mode tile accumulation: writes every cell of the G x G grid, or
// (skip_empty, f32 tap-table path) every cell of the tiles holding entries
// -- for a consumer that reads the bin counts (fft_grid_rows_cols). With
// accumulate (one batch of a call split into batches), the tiles holding
// entries are ADDED to the grid and nothing else is touched.
template<typename T>
int scatter(const EsParams<T>& p, const BucketScratch& s, uint32_t n_items,
        T* grid, hipStream_t stream, bool skip_empty = false,
        bool accumulate = false);

// 3-D, f32, W <= 8: planes p.plane .. p.plane + nplanes - 1 (into
// grids[0..nplanes), 2 <= nplanes <= planes_per_pass(p)) in one tile-kernel
// pass (skip_empty as scatter; no accumulate form).
template<typename T>
int planes_per_pass(const EsParams<T>& p);
template<typename T>
int scatter_planes(const EsParams<T>& p, const BucketScratch& s,
        uint32_t n_items, T* const* grids, int nplanes, hipStream_t stream,
        bool skip_empty);

// Degrid-mode tile gather: vis[idx] += sum_taps grid * kernel.
template<typename T>
int gather(const EsParams<T>& p, const BucketScratch& s, uint32_t n_items,
        const T* grid, T* vis, hipStream_t stream);

// Image-plane kernels. image N x N (real), grid G x G complex (interleaved).
// conv_corr: [N/2+1] normalised separable correction; quad_*: Gauss-Legendre
// tables (kQuadratureBound entries); norm: C(0).
template<typename T>
struct ImageParams
{
    int N;
    int G;
    int support;
    int do_w;
    T pixel_size;
    T norm;
    T inv_w_scale;
    T min_plane_w;
    const T* conv_corr;
    const T* quad_kernel;
    const T* quad_nodes;
    const T* quad_weights;
};

// 2-D grid path: dirty = (dirty + checker * Re(layer centre)) * corr.
template<typename T>
int screen_corr_2d(const ImageParams<T>& ip, const T* layer, T* dirty,
        hipStream_t stream);

// 3-D grid path, per plane: dirty += checker * Re(layer * phasor(w)).
template<typename T>
int screen_accumulate(const ImageParams<T>& ip, int plane, const T* layer,
        T* dirty, hipStream_t stream);

// dirty *= 1 / correction (2-D or 3-D correction), in place.
template<typename T>
int apply_correction(const ImageParams<T>& ip, T* dirty, hipStream_t stream);

// Degrid path: grid (all G x G cells) = centre: checker * dirty * phasor(w)
// (phasor = 1 in 2-D), zero elsewhere. If correct_in_place, the image is
// first multiplied by 1/correction and written back (2-D fused form).
template<typename T>
int reverse_screen(const ImageParams<T>& ip, int plane, T* dirty,
        bool correct_in_place, T* grid, hipStream_t stream);

} // namespace sdp_es

#endif
