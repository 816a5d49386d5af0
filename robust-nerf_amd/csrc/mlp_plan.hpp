// Layout plan of the fused NeRF MLP (reference noisy_src/model.py:83-221).
//
// Everything the host entry points and the kernels agree on lives here:
//   * the flat fp32 parameter layout (nn.Module.parameters() order),
//   * the packed MFMA fragment images of W (forward) and W^T (backward),
//   * the "saved" activations written by a training forward, and
//   * the backward workspace (per-layer pre-activation gradients dz and the
//     dW partial slabs).
//
// Sample tiles: 32 samples per tile (one MFMA column block).  Saved/workspace
// tensors are tile-blocked and feature-major: element (sample m, feature f)
// of a tensor with F (padded) features lives at  tile*F*32 + f*32 + (m%32),
// so the dW GEMM, whose reduction runs over samples, loads 16-byte operand
// fragments directly.  ReLU masks are bitmasks in accumulator-register order.
#pragma once

#include <cstdint>

#include "nerf_hip.h"

namespace nr {

constexpr int kHidden = 256;           // ModelConfig.hidden_dim supported by the kernels
constexpr int kHB = kHidden / 32;      // hidden feature blocks
constexpr int kMaxTrunk = 16;          // num_hidden_layers upper bound
constexpr int kMaxMfmaLayers = kMaxTrunk + 2;  // trunk + feature + dir
constexpr int kFragBytes = 1024;       // one wave-wide 16-B-per-lane operand fragment
constexpr int kMaxJobs = kMaxTrunk + 4;  // dW jobs: trunk + feat + dir + sigma + rgb
constexpr int kMaxSeg = 2;

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
};

// A dW job: gradient of one linear layer (heads included) from the saved
// input activations and the workspace dz.
struct DwJob {
    int layer;                 // index into MlpPlan::lin (sigma/rgb heads: kSigma/kRgb)
    int dz_tensor;             // workspace tensor holding dz (feature-major, F = NBz*32)
    int dz_row0;               // first dz row of this job inside that tensor (heads block)
    int rows;                  // valid output rows (out features)
    int NB;                    // output blocks computed
    int nin;                   // number of input tensors (segments)
    int in_tensor[kMaxSeg];    // saved tensor ids per segment
    int in_blocks[kMaxSeg];    // 32-blocks per segment
    int KB;                    // total input blocks
    int64_t slab_off;          // float offset of this job's slab (per chunk: NB*32*(KB*32+1))
};

// Saved tensor ids (training forward) and workspace tensor ids (backward).
enum SavedId { SV_XENC = 0, SV_H0 = 1 /* .. SV_H0+n_layers-1 */ };
enum WsId { WS_DZ0 = 0 /* dz of trunk i: WS_DZ0+i; then feat, dir, heads */ };

struct MlpPlan {
    int L, Ld, n_layers, use_vd, prec;
    uint32_t skips;
    int pos_dim, dir_dim, XB, DB;
    int64_t param_count;
    int n_lin;                        // trunk + feat + dir (MFMA layers)
    LinearDesc lin[kMaxMfmaLayers];   // [0, n_layers) trunk, n_layers feat, n_layers+1 dir
    int64_t sig_w, sig_b, rgb_w, rgb_b;
    int64_t packed_bytes;
    int esize;                        // bytes per saved/workspace element (2 bf16, 4 fp32)
    // saved tensors
    int n_saved;                      // xenc, h0..h_{n-1}, feat, denc, hc
    int sv_feat, sv_denc, sv_hc;
    int sv_F[kMaxTrunk + 4];          // padded features per saved tensor
    int n_mask;                       // mask words: trunk layers + hc
    // workspace tensors
    int n_ws;                         // dz_0..dz_{n-1}, dz_feat, dz_dir, dz_heads
    int ws_feat, ws_dir, ws_heads;
    int ws_F[kMaxTrunk + 3];
    // dW jobs
    int n_jobs;
    DwJob job[kMaxJobs];
    int64_t slab_floats_per_chunk;
};

inline bool is_skip(const MlpPlan& p, int i) { return (p.skips >> i) & 1u; }

// Builds the plan; returns false (with *why set) for unsupported configs.
bool make_plan(const NrMlpConfig* cfg, MlpPlan* p, const char** why);

// Byte sizes / offsets that depend on the number of samples.
struct MlpSizes {
    int64_t tiles;
    int64_t saved_off[kMaxTrunk + 4];  // bytes
    int64_t mask_off;                  // bytes
    int64_t saved_bytes;
    int64_t ws_off[kMaxTrunk + 3];     // bytes
    int chunks;                        // dW split over sample tiles
    int64_t slab_off;                  // bytes
    int64_t ws_bytes;
};

MlpSizes make_sizes(const MlpPlan& p, int64_t M);

}  // namespace nr
