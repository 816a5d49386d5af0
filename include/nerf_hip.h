/*
 * nerf_hip.h — C ABI of the MI355X (gfx950) NeRF training hot path.
 *
 * This is the drop-in boundary beneath the Python host package `noisy_src`
 * (robust-nerf_amd/noisy_src), which mirrors the reference package
 * ShawnnnLiu/Robust-NeRF `noisy_src/` (rays.py, model.py, rendering.py,
 * train_pose_opt.py, data_pose_opt.py).  The reference is pure PyTorch and has
 * no FFI of its own; every entry point below replaces the reference function
 * cited beside it, and the ctypes binding a maintainer would add is shown in
 * INTEGRATION.md.
 *
 * Contract shared by every entry point:
 *   - returns NR_OK (0) on success, a positive hipError_t on a HIP runtime
 *     failure, or NR_EARG on an argument error; nr_last_error() describes it;
 *   - all array pointers are CALLER-OWNED DEVICE pointers (PyTorch caching
 *     allocator); fp32 arrays are dense row-major exactly like the torch
 *     tensors of the reference ((..., 3) arrays are AoS);
 *   - no entry point allocates, frees or synchronises: kernels are enqueued on
 *     `stream` (the caller's torch.cuda.current_stream()), so calls can be
 *     captured into a hipGraph;
 *   - "nullable" pointers may be NULL to skip an optional input/output.
 */
#ifndef NERF_HIP_H
#define NERF_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define NR_OK 0
#define NR_EARG (-22)

typedef void* nr_stream_t; /* a hipStream_t */

/* ---- library ----------------------------------------------------------- */
const char* nr_last_error(void);
int nr_abi_version(void);
/* Toolchain probe (no reference counterpart): out[i] = value + i. */
int nr_probe_fill(float* out, int n, float value, nr_stream_t stream);
/* Diagnostic: one MFMA tile, kind 0 = bf16 32x32x16 (A 32x16, B 16x32),
 * kind 1 = f32 32x32x2 (A 32x2, B 2x32); D (32,32) row-major = A @ B. */
int nr_probe_mfma(int kind, const float* A, const float* B, float* D,
                  nr_stream_t stream);

/* ---- A1: get_ray_directions  (noisy_src/rays.py:17-64) ------------------
 * dirs (H,W,3): ((i-cx)/focal, -(j-cy)/focal, -1), meshgrid indexing='xy'. */
int nr_ray_directions(int H, int W, float focal, float cx, float cy,
                      float* dirs, nr_stream_t stream);

/* ---- A2: get_rays  (noisy_src/rays.py:67-99) -----------------------------
 * dirs (N,3), c2w (4,4) -> rays_o (N,3) = t, rays_d (N,3) = normalize(R d). */
int nr_get_rays(const float* dirs, const float* c2w, int64_t N,
                float* rays_o, float* rays_d, nr_stream_t stream);
/* Backward of get_rays (the reference's is differentiable in c2w and dirs):
 * g_c2w (4,4) ACCUMULATED (caller zeroes), rows 0..2 / cols 0..3 (R and t);
 * g_dirs (N,3) OVERWRITTEN, nullable; g_rays_o / g_rays_d nullable (not both;
 * g_dirs needs g_rays_d).  Fixed-order reduction over the N rays through
 * nr_get_rays_bwd_workspace_bytes() of scratch.                             */
int64_t nr_get_rays_bwd_workspace_bytes(void);
int nr_get_rays_bwd(const float* dirs, const float* c2w, int64_t N,
                    const float* g_rays_o, const float* g_rays_d,
                    float* g_dirs, float* g_c2w, void* workspace,
                    nr_stream_t stream);

/* ---- A3: PixelDataset.get_rays_from_pixels  (noisy_src/data_pose_opt.py:83-148,
 *          PixelSampler.get_rays_for_batch :200-223) ---------------------
 * One pass over the batch, no per-image host loop.  img_idx (B,) int64,
 * pix (B,2) fp32 (u,v) pixel coords, poses (n_img,4,4) indexed by img_idx.
 * Validating mode: bad_index (nullable, one device int the caller zeroes) is
 * set to 1 when any img_idx lies outside [0, n_img) -- the reference's
 * poses[idx] raises IndexError there (data_pose_opt.py:105-148); the entry
 * point stays asynchronous (graph-capturable), so the host wrapper reads the
 * flag and raises.  Such rays come out NaN either way.                      */
int nr_rays_from_pixels_fwd(const int64_t* img_idx, const float* pix,
                            const float* poses, int n_img, int H, int W,
                            float focal, int B, float* rays_o, float* rays_d,
                            int* bad_index, nr_stream_t stream);
/* Backward: g_poses (n_img,4,4) must be zeroed by the caller; it receives
 * dL/dposes summed over the pixels of each image (g_rays_d nullable).  One
 * workgroup per image sums its rays in a fixed order: no atomics, the result is
 * bit-identical from run to run.  Rays whose img_idx is outside [0, n_img)
 * contribute nothing (the forward writes NaN rays for them); callers that take
 * indices from outside validate them with nr_check_index_range.            */
int nr_rays_from_pixels_bwd(const int64_t* img_idx, const float* pix,
                            const float* poses, int n_img, int H, int W,
                            float focal, int B, const float* g_rays_o,
                            const float* g_rays_d, float* g_poses,
                            nr_stream_t stream);
/* flag[0] = 1 if any idx[i] (i < n) lies outside [0, limit); flag untouched
 * otherwise (caller zeroes it).  Validation for host wrappers that receive
 * indices from a user (the reference raises IndexError on them).            */
int nr_check_index_range(const int64_t* idx, int n, int limit, int* flag,
                         nr_stream_t stream);

/* ---- A4: CameraPoseParameters.get_poses  (noisy_src/train_pose_opt.py:122-226)
 * poses_out[i] = [[R_delta(rot[idx_i]) @ R_init[idx_i], t_init[idx_i] + trans[idx_i]],
 *                 [0 0 0 1]], with the reference's theta < 1e-6 -> I rule
 * (train_pose_opt.py:143-144,161).  rot / trans / indices nullable.        */
int nr_se3_poses_fwd(const float* init_poses, const float* rot_deltas,
                     const float* trans_deltas, const int64_t* indices, int n,
                     float* poses_out, nr_stream_t stream);
/* Backward of the above.  g_rot / g_trans (n_poses,3) are ACCUMULATED (indices
 * may repeat; each pose sums its rows in row order, deterministically); the
 * caller zeroes them.  At theta < 1e-6 dL/drot is exactly 0, as in the
 * reference (the torch.where blocks the gradient). fixed_small_angle != 0
 * selects the first-order small-angle Jacobian instead (non-default flag).  */
int nr_se3_poses_bwd(const float* init_poses, const float* rot_deltas,
                     const int64_t* indices, int n, int n_poses,
                     const float* g_poses,
                     int fixed_small_angle, float* g_rot, float* g_trans,
                     nr_stream_t stream);

/* ---- batch assembly: RaySampler  (noisy_src/data.py:264-321) -----------
 * out_*[b] = table_*[idx[b]] for the (n_rays,3) ray table (rays_o, rays_d,
 * colors) in one launch; idx outside [0, n_rays) gives NaN rows and, in the
 * validating mode (bad_index non-NULL, caller-zeroed device int), sets
 * *bad_index = 1 for the host wrapper to raise IndexError (torch indexing in
 * the reference's data.py:305-309 raises).                                   */
int nr_gather_rays(const int64_t* idx, int64_t n_rays, int B,
                   const float* rays_o, const float* rays_d, const float* colors,
                   float* out_o, float* out_d, float* out_rgb, int* bad_index,
                   nr_stream_t stream);

/* ---- A5: sample_along_rays  (noisy_src/rays.py:145-210) ------------------
 * z (B,N); pts (B,N,3) nullable.  t_rand (B,N) nullable -> no perturbation.
 * viewdirs (B*N,3) nullable: rays_d / |rays_d| per sample (rendering.py:165), as
 * nr_expand_viewdirs writes it.                                               */
int nr_stratified_sample(const float* rays_o, const float* rays_d,
                         const float* t_rand, float near_, float far_,
                         int lindisp, int B, int N, float* z_vals, float* pts,
                         float* viewdirs, nr_stream_t stream);

/* ---- A6: PositionalEncoding.forward  (noisy_src/model.py:58-80) ----------
 * x (M,C) -> out (M, C*(include_input + 2L)) laid out [x | sin f0x | cos f0x | ...]. */
int nr_positional_encoding(const float* x, int64_t M, int C, int num_freqs,
                           int include_input, int log_sampling, float* out,
                           nr_stream_t stream);
int nr_positional_encoding_bwd(const float* x, int64_t M, int C, int num_freqs,
                               int include_input, int log_sampling,
                               const float* g_out, float* g_x,
                               nr_stream_t stream);

/* ---- A9: sample_pdf  (noisy_src/rays.py:213-279) -------------------------
 * bins (B,Nb), weights (B,Nb-1), u (B,Ns) nullable -> det=True linspace(0,1).
 * samples (B,Ns) in the order of u.                                         */
int nr_sample_pdf(const float* bins, const float* weights, const float* u,
                  int B, int Nb, int Ns, float* samples, nr_stream_t stream);

/* ---- A10: sample_hierarchical  (noisy_src/rays.py:282-333) ---------------
 * z_coarse (B,Nc), w_coarse (B,Nc) -> z_fine (B,Nc+Nf) = sort(cat(z, sample_pdf(
 * mid(z), w[:,1:-1], Nf, det))), pts_fine (B,Nc+Nf,3) nullable.  u nullable=det.
 * viewdirs (B*(Nc+Nf),3) nullable, as in nr_stratified_sample.               */
int nr_sample_hierarchical(const float* rays_o, const float* rays_d,
                           const float* z_coarse, const float* w_coarse,
                           const float* u, int B, int Nc, int Nf,
                           float* z_fine, float* pts_fine, float* viewdirs,
                           nr_stream_t stream);

/* ---- A8: raw2outputs  (noisy_src/rendering.py:20-116) --------------------
 * rgb (B,S,3), sigma (B,S), z (B,S), rays_d (B,3), sigma_noise (B,S) nullable
 * (already scaled by raw_noise_std) -> rgb_map (B,3), depth (B), acc (B),
 * weights (B,S).                                                           */
int nr_composite_fwd(const float* rgb, const float* sigma, const float* z,
                     const float* rays_d, const float* sigma_noise, int B,
                     int S, int white_bg, float* rgb_map, float* depth_map,
                     float* acc_map, float* weights, nr_stream_t stream);
/* Backward: g_depth / g_acc / g_weights nullable (zero); g_rays_d nullable
 * (ACCUMULATED: dL/drays_d through dists * |rays_d|). */
int nr_composite_bwd(const float* rgb, const float* sigma, const float* z,
                     const float* rays_d, const float* sigma_noise, int B,
                     int S, int white_bg, const float* g_rgb_map,
                     const float* g_depth, const float* g_acc,
                     const float* g_weights, float* g_rgb, float* g_sigma,
                     float* g_rays_d, nr_stream_t stream);

/* ---- A7: NeRF MLP  (noisy_src/model.py:83-221) ---------------------------
 * Parameters live in one flat fp32 buffer in nn.Module.parameters() order:
 * pts_linears.{0..L-1}.{weight,bias}, sigma_linear, feature_linear,
 * dir_linear, rgb_linear (weights (out,in) row-major, as nn.Linear).       */
typedef struct NrMlpConfig {
    int pos_freqs;      /* ModelConfig.pos_freqs (10)          */
    int dir_freqs;      /* ModelConfig.dir_freqs (4)           */
    int hidden;         /* ModelConfig.hidden_dim (256)        */
    int n_layers;       /* ModelConfig.num_hidden_layers (8)   */
    uint32_t skip_mask; /* bit i set <=> i in ModelConfig.skips */
    int use_view_dirs;  /* ModelConfig.use_view_dirs (1)       */
    int precision;      /* NR_PREC_FP32 / NR_PREC_BF16         */
    int dense_backward; /* 0: the backward skips 32-sample tiles whose incoming
                           gradient (g_rgb, g_sigma) is exactly zero; nonzero:
                           every tile (the dense reference form)          */
} NrMlpConfig;

#define NR_PREC_FP32 0
#define NR_PREC_BF16 1
#define NR_PREC_FP16 2  /* cfg #5: fp16 MFMA operands, fp32 accumulate, 2^14 backward loss scale */

/* Sizes (bytes unless stated).  M = number of samples. */
int64_t nr_mlp_param_count(const NrMlpConfig* cfg);
int64_t nr_mlp_packed_bytes(const NrMlpConfig* cfg);
int64_t nr_mlp_saved_bytes(const NrMlpConfig* cfg, int64_t M);
int64_t nr_mlp_workspace_bytes(const NrMlpConfig* cfg, int64_t M);

/* Re-pack the flat fp32 parameters into the MFMA fragment images used by the
 * forward (W) and backward (W^T) kernels.  Call after every optimizer step. */
int nr_mlp_pack(const NrMlpConfig* cfg, const float* params, void* packed,
                nr_stream_t stream);

/* Forward: x (M,3) positions, d (M,3) view directions -> rgb (M,3) in [0,1],
 * sigma (M) >= 0.  saved (nr_mlp_saved_bytes) nullable: inference only.   */
int nr_mlp_forward(const NrMlpConfig* cfg, const void* packed,
                   const float* params, const float* x, const float* d,
                   int64_t M, float* rgb, float* sigma, void* saved,
                   nr_stream_t stream);

/* Backward: g_rgb (M,3), g_sigma (M) -> g_params (flat, OVERWRITTEN),
 * g_x (M,3) / g_d (M,3) nullable (OVERWRITTEN).  Needs the forward's
 * `saved` and rgb/sigma outputs, and nr_mlp_workspace_bytes of workspace.
 * Runs the split form: nr_mlp_backward_dx, _dw, _reduce.                    */
int nr_mlp_backward(const NrMlpConfig* cfg, const void* packed,
                    const float* params, const float* x, const float* d,
                    int64_t M, const float* rgb, const float* sigma,
                    const void* saved, const float* g_rgb,
                    const float* g_sigma, float* g_params, float* g_x,
                    float* g_d, void* workspace, nr_stream_t stream);

/* The three stages of nr_mlp_backward, callable separately (per-kernel timing):
 * dx: the list of ACTIVE 32-sample tiles (any nonzero g_rgb / g_sigma entry;
 * every tile with cfg->dense_backward) and the dz of every layer for them into
 * the workspace (+ g_x / g_d, zero for inactive samples); dw: per-chunk dW/db
 * slabs from the saved activations and dz of the active tiles, split over the
 * chunks in list order; reduce: slabs -> g_params (chunk order, deterministic).
 * A tile whose incoming gradient is exactly zero has dz == 0 in every layer, so
 * skipping it drops only exact-zero terms; when every tile is active the result
 * is bit-identical to the dense form.  Same arguments and workspace as
 * nr_mlp_backward; dw must follow dx on the same workspace.                 */
int nr_mlp_backward_dx(const NrMlpConfig* cfg, const void* packed,
                       const float* params, const float* x, const float* d,
                       int64_t M, const float* rgb, const float* sigma,
                       const void* saved, const float* g_rgb,
                       const float* g_sigma, float* g_x, float* g_d,
                       void* workspace, nr_stream_t stream);
int nr_mlp_backward_dw(const NrMlpConfig* cfg, int64_t M, const void* saved,
                       void* workspace, nr_stream_t stream);
int nr_mlp_backward_reduce(const NrMlpConfig* cfg, int64_t M,
                           const void* workspace, float* g_params,
                           nr_stream_t stream);
/* Byte offset in the workspace of the uint32 count of active tiles that
 * nr_mlp_backward_dx wrote (of ceil(M / 32)), or -1: the work the backward ran. */
int64_t nr_mlp_active_tiles_offset(const NrMlpConfig* cfg, int64_t M);

/* ---- A13: optimizer tail  (noisy_src/train.py:112-117, train_pose_opt.py:398-409)
 * Sum of squares of n fp32 values added into *acc (device scalar, caller-zeroed):
 * the squared global norm of torch.nn.utils.clip_grad_norm_.  A fixed-shape
 * two-pass reduction (deterministic) through nr_sumsq_workspace_bytes() of
 * caller-owned scratch; calls on one stream may share the scratch.          */
int64_t nr_sumsq_workspace_bytes(void);
int nr_sumsq(const float* x, int64_t n, float* acc, void* workspace,
             nr_stream_t stream);
/* torch.optim.Adam (amsgrad=False, maximize=False, weight_decay=0) on a flat
 * buffer: grads are first scaled by clip = min(1, max_norm / (sqrt(*sumsq)
 * + 1e-6)) when sumsq != NULL (torch.nn.utils.clip_grad_norm_), lr is read
 * from the host (LambdaLR already applied), step is the 1-based Adam step. */
int nr_adam_step(float* params, float* grads, float* exp_avg,
                 float* exp_avg_sq, int64_t n, double lr, double beta1,
                 double beta2, double eps, int64_t step, const float* sumsq,
                 float max_norm, nr_stream_t stream);

/* The fused optimizer tail of one training step (train.py:112-117: clip_grad_norm_
 * + optimizer.step(); train_pose_opt.py:398-409 with one clip per network), in two
 * launches however many flat buffers it covers, and without the re-pack after it:
 *
 * nr_sumsq_partials: the nr_sumsq_workspace_bytes() of fixed-order partial sums of
 * squares over the concatenation of nspan (<= 8) fp32 buffers (one clip group),
 * written to `partials` (OVERWRITTEN; no caller-zeroed accumulator).          */
int nr_sumsq_partials(const float* const* xs, const int64_t* ns, int nspan,
                      float* partials, nr_stream_t stream);
/* One flat buffer of nr_adam_multi.  sumsq_partials (nullable: no clip) is the
 * nr_sumsq_partials output of the buffer's clip group, whose grads are scaled by
 * min(1, max_norm / (sqrt(sum) + 1e-6)) as nr_adam_step does.  pack_table
 * (nullable) refreshes the MFMA images `packed` of an MLP whose flat parameters
 * are `params`: every updated parameter is written, converted as nr_mlp_pack
 * converts it, to each image position the table lists, so `packed` equals
 * nr_mlp_pack(params) afterwards when it did before (bit-identical).          */
typedef struct NrAdamSpan {
    float* params;
    float* grads;
    float* exp_avg;
    float* exp_avg_sq;
    int64_t n;
    const float* sumsq_partials;
    float max_norm;
    const uint32_t* pack_table;
    void* packed;
} NrAdamSpan;
/* torch.optim.Adam over nspan (<= 8) buffers of one param group (same lr and
 * 1-based step), one launch.  sched (nullable, device): {lr / (1 - beta1^step),
 * sqrt(1 - beta2^step)} as fp32, read by the kernel instead of the host lr/step,
 * so a captured hipGraph of the step can be replayed with the schedule advanced
 * by a 8-byte copy (lr / step then only validate).                          */
int nr_adam_multi(const NrAdamSpan* spans, int nspan, double lr, double beta1,
                  double beta2, double eps, int64_t step, const float* sched,
                  nr_stream_t stream);
/* The destination table of an MLP's packed images for nr_adam_multi: for each
 * of the nr_mlp_param_count() flat parameters, 3 slots of (kind << 29 | byte
 * offset in packed), slot-major (table[s * n + i]); built once per config by
 * the index maps of nr_mlp_pack itself.                                     */
int64_t nr_mlp_pack_table_bytes(const NrMlpConfig* cfg);
int nr_mlp_pack_table(const NrMlpConfig* cfg, uint32_t* table,
                      nr_stream_t stream);

/* ---- per-ray glue used by render_rays (rendering.py:119-240) ------------ */
/* viewdirs = d/|d| broadcast to every sample: out (B*S,3). */
int nr_expand_viewdirs(const float* rays_d, int B, int S, float* out,
                       nr_stream_t stream);
/* g_rays_o[b] += sum_s g_pts[b,s]; g_rays_d[b] += sum_s g_pts[b,s]*z[b,s]
 * (pts = o + d z, rays.py:208/331).  Either output nullable. */
int nr_pts_bwd(const float* g_pts, const float* z, int B, int S,
               float* g_rays_o, float* g_rays_d, nr_stream_t stream);
/* g_rays_d[b] += d(viewdir)/d(rays_d)^T sum_s g_viewdirs[b,s] (rendering.py:165). */
int nr_viewdirs_bwd(const float* rays_d, const float* g_viewdirs, int B,
                    int S, float* g_rays_d, nr_stream_t stream);
/* loss = mean((pred - target)^2) over B*3; g_pred = 2/(3B) (pred-target)*scale;
 * loss_out (device scalar, OVERWRITTEN) may be NULL. */
int nr_mse_fwd_bwd(const float* pred, const float* target, int B, float scale,
                   float* loss_out, float* g_pred, nr_stream_t stream);
/* The training form of raw2outputs + the MSE loss (rendering.py:20-116 then
 * train.py:89/98): the composite forward (outputs as nr_composite_fwd), the loss
 * (device scalar, OVERWRITTEN) against target (B,3), and the backward of
 * grad_scale * loss (g_rgb, g_sigma OVERWRITTEN; g_rays_d nullable, ACCUMULATED) in one
 * wave per ray -- gradients bit-identical to nr_composite_fwd, nr_mse_fwd_bwd and
 * nr_composite_bwd in sequence.  ticket (nullable): a device uint32 that is 0 before
 * the call and is left 0; with it (and B <= 1024) the launch's last workgroup sums the
 * loss, otherwise a second launch does.  Calls sharing a ticket must not run concurrently.
 * workspace: nr_composite_mse_workspace_bytes(B).                                 */
int64_t nr_composite_mse_workspace_bytes(int B);
int nr_composite_mse(const float* rgb, const float* sigma, const float* z,
                     const float* rays_d, const float* sigma_noise,
                     const float* target, int B, int S, int white,
                     float grad_scale, float* rgb_map, float* depth_map,
                     float* acc_map, float* weights, float* loss, float* g_rgb,
                     float* g_sigma, float* g_rays_d, uint32_t* ticket,
                     void* workspace, nr_stream_t stream);

#ifdef __cplusplus
}
#endif

#endif /* NERF_HIP_H */
