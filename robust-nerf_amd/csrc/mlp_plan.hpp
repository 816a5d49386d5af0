// Layout plan of the fused NeRF MLP (reference noisy_src/model.py:83-221).
//
// Everything the host entry points and the kernels agree on lives here:
//   * the flat fp32 parameter layout (nn.Module.parameters() order),
//   * the packed MFMA fragment images of W (forward) and W^T (backward),
//     stored chunk-major: one chunk = every row block of one 32-wide k block,
//     i.e. exactly what the kernels stream through LDS per step, each
//     direction's images laid out in its stream order;
//   * fp32 vectors (biases, w_sigma, W_rgb) in accumulator-register order;
//   * the activations saved by a training forward and the per-layer
//     pre-activation gradients dz written by the backward, both stored as
//     MFMA B-operand images: per 32-sample tile and 32-feature block, FPB
//     wave-wide 1-KB fragments (lane L = sample + 32*h holds 16 B), so every
//     store is a fully coalesced 1-KB wave write.
// ReLU masks are bitmasks in accumulator-register order (16 B per lane per layer).
#pragma once

#include <cstdint>

#include "nerf_hip.h"

namespace nr {

constexpr int kHidden = 256;           // ModelConfig.hidden_dim supported by the kernels
constexpr int kHB = kHidden / 32;      // hidden feature blocks
constexpr int kMaxTrunk = 16;          // num_hidden_layers upper bound
constexpr int kMaxMfmaLayers = kMaxTrunk + 2;  // trunk + feature + dir
constexpr int kFragBytes = 1024;       // one wave-wide 16-B-per-lane operand fragment
constexpr int kScratchTiles = 64;  // dX waves without an active tile spread their stores over these
constexpr int kSegTiles = 256;  // tiles per segment of the active-tile list
constexpr int kMaxJobs = kMaxTrunk + 8;  // dW jobs: x-jobs + trunk h-jobs + feat + heads + dir
constexpr int kMaxSeg = 2;
constexpr int kMaxJobSeg = 4;            // tensors on either side of a dW job
constexpr int kMaxRed = kMaxTrunk + 4;    // reduce ranges: trunk, feat, sigma, rgb, dir
// dW staging: each of the 8 waves issues at most this many 1-KB LDS-DMA pieces
// per tile, so a job's (NBz + KB) * FPB blocks must not exceed 8x it
__host__ __device__ constexpr int dw_max_pieces(bool k16) { return k16 ? 6 : 10; }

// One input segment of a linear layer: columns [col0, col0+width) of W,
// occupying ceil(width/32) consecutive 32-wide input blocks.
struct Seg {
    int col0, width, blocks;
};

struct LinearDesc {
    int64_t w_off, b_off;  // offsets into the flat parameter buffer (floats)
    int out, in;           // nn.Linear shape (out, in)
    int NB, KB;            // output / input 32-blocks (padded)
    int nseg;
    Seg seg[kMaxSeg];
    int64_t pk_fwd, pk_bwd;  // byte offsets of the W / W^T fragment images
    int64_t pk_bwdr;         // 16-bit: row-block-major W^T image of the h (feat) input rows (dX chain)
    int64_t vb;              // byte offset of the bias vector image (accumulator order)
};

// A tensor range of a dW job: `blocks` consecutive 32-feature blocks of
// saved (is_ws = 0) or workspace (is_ws = 1) tensor `tensor`.
struct DwSeg {
    int is_ws, tensor, blocks;
};

// One wave's share of a dW job: dz row blocks [row0, row0+np) x input column
// blocks [col0, col0+nq) (np <= kDwMaxP, nq <= kDwMaxQ), plus the bias partial
// sums of those dz rows when bias != 0.
constexpr int kDwMaxWaves = 8;
constexpr int kDwMaxP = 5, kDwMaxQ = 2;
struct DwWave {
    int row0, np, col0, nq, bias;
};

// A dW job: products dz^T . in over the tiles of one chunk, for the 32x32 blocks
// its waves list, inside an NBz x KB grid (dz segments stacked as rows, input
// segments as columns; every tensor is staged once per tile).  Output slab per
// chunk: (NBz*32) x (KB*32 + 1) floats, the last column holding the bias partial
// sums of the dz rows; blocks no wave lists are never written or read.
struct DwJob {
    int ndz, nin;
    DwSeg dz[kMaxJobSeg], in[kMaxJobSeg];
    int NBz, KB;
    int64_t slab_off;  // float offset of this job's slab inside one chunk's slab set
    int nwaves;
    DwWave w[kDwMaxWaves];
};

// Saved tensor ids (training forward) and workspace tensor ids (backward).
enum SavedId { SV_XENC = 0, SV_H0 = 1 /* .. SV_H0+n_layers-1 */ };
enum WsId { WS_DZ0 = 0 /* dz of trunk i: WS_DZ0+i; then feat, dir, heads */ };

// Per-parameter-range map for the slab reduction: W (rows x in, at w_off) takes
// its column segments from job slabs (slab row slab_row0 + r, column
// slab_col0 + c - col0); the bias (b_off, rows) from job bjob's bias column.
struct RedSeg {
    int col0, width, job, slab_row0, slab_col0;
};
struct ReduceRange {
    int rows, in;
    int64_t w_off, b_off;
    int nseg;
    RedSeg seg[kMaxSeg];
    int bjob, brow0;
};

struct MlpPlan {
    int L, Ld, n_layers, use_vd, prec;
    int dense_bwd;                    // NrMlpConfig.dense_backward: every tile through the backward
    uint32_t skips;
    int pos_dim, dir_dim, XB, DB;
    int64_t param_count;
    int n_lin;                        // trunk + feat + dir (MFMA layers)
    LinearDesc lin[kMaxMfmaLayers];   // [0, n_layers) trunk, n_layers feat, n_layers+1 dir
    int64_t sig_w, sig_b, rgb_w, rgb_b;
    int64_t packed_bytes;
    int64_t vsig, vrgb;               // byte offsets of the w_sigma / W_rgb vector images
    int64_t vhead;                    // 16-bit forward: w_sigma then the 3 W_rgb rows as vector images (3 KB)
    int esize;                        // bytes per saved/workspace element (2 bf16, 4 fp32)
    int fpb;                          // 1-KB fragments per 32x32 block (2 bf16, 4 fp32)
    // saved tensors
    int n_saved;                      // xenc, h0..h_{n-1}, feat, denc, hc
    int sv_feat, sv_denc, sv_hc;
    int sv_F[kMaxTrunk + 4];          // padded features per saved tensor
    int n_mask;                       // mask words: trunk layers + hc
    // workspace tensors
    int n_ws;                         // dz_0..dz_{n-1}, dz_feat, dz_dir, dz_heads
    int ws_feat, ws_dir, ws_heads;
    int ws_F[kMaxTrunk + 3];
    // dW jobs and the reduction map
    int n_jobs;
    DwJob job[kMaxJobs];
    int64_t slab_floats_per_chunk;
    int n_red;
    ReduceRange red[kMaxRed];
};

inline bool is_skip(const MlpPlan& p, int i) { return (p.skips >> i) & 1u; }

// Builds the plan; returns false (with *why set) for unsupported configs.
bool make_plan(const NrMlpConfig* cfg, MlpPlan* p, const char** why);

// Byte sizes / offsets that depend on the number of samples.
struct MlpSizes {
    int64_t tiles;
    int64_t tiles_alloc;  // tiles rounded up to whole 16-tile groups (every fwd wave may store its tile),
                          // then kScratchTiles scratch tiles (dX waves without a tile store there)
    int64_t saved_off[kMaxTrunk + 4];  // bytes
    int64_t mask_off;                  // bytes
    int64_t saved_bytes;
    int64_t ws_off[kMaxTrunk + 3];     // bytes
    int chunks;                        // dW split over sample tiles
    int job_chunks[kMaxJobs];          // dW workgroups of each job (16-bit: all = chunks; fp32: by cost)
    int max_chunks;                    // per-chunk slab sets allocated (the largest job_chunks)
    int64_t slab_off;                  // bytes
    int64_t nseg;                      // segments of kSegTiles tiles
    // bytes: tile flags (u8, nseg * kSegTiles); 64-tile block counts; the dW list; its length
    int64_t flags_off, blkcnt_off, dwlist_off, count_off;
    int64_t ws_bytes;
};

MlpSizes make_sizes(const MlpPlan& p, int64_t M);

}  // namespace nr
