/* mzba.h — C ABI of the MI355X (gfx950) MuZero-Breakout acting path (libmzba.so).
 *
 * Plain pointers (device memory unless noted) and sizes; `stream` is a hipStream_t
 * (torch's current stream from Python). Every function returns 0 on success, a
 * negative code for an invalid argument, or the positive hipError_t of a failed
 * launch. Work is stream-ordered and never synchronises the host, so every call is
 * HIP-graph capturable. Each entry point names the reference interface it replaces.
 * Numerics and layouts: DESIGN.md.
 */
#ifndef MZBA_H
#define MZBA_H
#include <stdint.h>
#include <hip/hip_runtime_api.h>

#ifdef __cplusplus
extern "C" {
#endif

/* ---- environment (environment/parallel_breakout.py) ---------------------------------- */

/* BreakoutEnvironment.reset (parallel_breakout.py:107-139). state f32 (B,3,H,W), ball_dx i64[B],
 * ball_dy f32[B]. Random draws from Philox(seed; env+env_offset, stream 0, episode, kind) or, when
 * params != NULL, int32 params[4][B] = (paddle offset, ball col, ball row offset, dx). */
int mzba_env_reset_planes(float* state, int64_t* ball_dx, float* ball_dy, int B, int H, int W, int paddle_width,
                          int brick_rows, uint64_t seed, int episode, int env_offset, const int32_t* params,
                          hipStream_t stream);

/* BreakoutEnvironment.step (parallel_breakout.py:158-254) + get_valid_actions (:141-155).
 * done (u8[B], torch.bool storage) is updated in place. rewards4 (HOST) = {paddle_hit, brick_hit,
 * game_lost, game_won}. *err |= 1 if an env does not hold exactly one ball (the reference raises). */
int mzba_env_step_planes(const float* state, float* next_state, const int64_t* action, uint8_t* done,
                         int64_t* ball_dx, float* ball_dy, float* reward, float* valid, int B, int H, int W,
                         int paddle_width, const float* rewards4, int32_t* err, hipStream_t stream);

/* RLSystem.convert_to_grayscale (train_torch.py:334-358): (B,3,H,W) -> (B,1,H,W) f32. */
int mzba_grayscale_planes(const float* state, float* gray, int B, int H, int W, hipStream_t stream);

/* Frame storage (reset / step / rep input / current frame): cur_src (u8[B], may be NULL) selects
 * single-write mode — a frame recorded into the history ring is not also copied to cur_frame;
 * cur_src[b] = 1 says env b's current frame is the ring's newest entry, 0 that it is cur_frame[b]
 * (a done env: history frozen, frame live). With cur_src = NULL cur_frame always holds it.
 * Compact env for the fused acting loop: same rules as mzba_env_step_planes on SoA scalars
 * (paddle col, ball x/y, dx, dy, done) + a brick bitmask (nw u64 words per env over the brick rows).
 * Reset also does _pad_initial_state (train_torch.py:313-332): frame-history ring filled with
 * g(s0) (L-1 frames of H*W u8 gray codes), action ring (L) filled with pad_action (0 for the acting
 * loop, 1 for run_test_simulation, train_torch.py:545), hist_len = 0. */
int mzba_env_reset_compact(int32_t* paddle, int32_t* bx, int32_t* by, int32_t* dx, float* dy, uint8_t* done,
                           uint64_t* bricks, int nw, uint8_t* cur_frame, uint8_t* cur_src, uint8_t* hist_frames,
                           uint8_t* hist_actions, int32_t* hist_len, int L, int B, int H, int W, int paddle_width,
                           int brick_rows, uint64_t seed, int episode, int env_offset, const int32_t* params,
                           int pad_action, hipStream_t stream);

/* One acting-loop env step (train_torch.py:201-209): step, render the u8 gray frame, push
 * (action, frame) into the history ring when the env is recorded (not prev_done; at the first
 * step prev_done aliases done, :179), and write the trajectory-sink row (rec_* may be NULL).
 * ctx (optional, graph replay): device int32[3] step context; when given, the sink row is
 * ctx[2] (rec_* are the (T,B,..) bases) and first_step = (ctx[2] == 0). */
/* rec_flags: 0 = record envs that were live before the step (the acting loop); bit 0 = record every
 * env, bit 1 = record env 0's action for every env (run_test_simulation, train_torch.py:594-598). */
int mzba_env_step_compact(int32_t* paddle, int32_t* bx, int32_t* by, int32_t* dx, float* dy, uint8_t* done,
                          uint64_t* bricks, int nw, const int64_t* action, float* reward, float* valid,
                          uint8_t* cur_frame, uint8_t* cur_src, uint8_t* hist_frames, uint8_t* hist_actions,
                          int32_t* hist_len, int L, uint8_t* rec_action, float* rec_reward, uint8_t* rec_mask, uint8_t* rec_frame,
                          int first_step, int B, int H, int W, int paddle_width, int brick_rows,
                          const float* rewards4, const int32_t* ctx, int rec_flags, hipStream_t stream);

/* Diagnostics: envs per workgroup of mzba_env_step_compact (0 = automatic). */
int mzba_env_set_block_envs(int E);

/* compact -> reference planes (B,3,H,W) f32. */
int mzba_compact_to_planes(const int32_t* paddle, const int32_t* bx, const int32_t* by, const uint8_t* done,
                           const uint64_t* bricks, int nw, float* planes, int B, int H, int W, int paddle_width,
                           int brick_rows, hipStream_t stream);

/* RLSystem._prepare_mcts_input + _encode_actions (train_torch.py:259-293) for all envs:
 * NHWC out [B][HW][Cs] (f32 or bf16): L-1 ring frames oldest first, the current frame, L action
 * planes a/3, zero padding to Cs. */
int mzba_build_rep_input(const uint8_t* cur_frame, const uint8_t* cur_src, const uint8_t* hist_frames,
                         const uint8_t* hist_actions, const int32_t* hist_len, int L, void* out, int out_bf16, int B,
                         int HW, int Cs, hipStream_t stream);

/* Every env's current frame [B][HW] u8 gray codes (for host readers: frame logging, tests). */
int mzba_env_current_frame(const uint8_t* cur_frame, const uint8_t* cur_src, const uint8_t* hist_frames,
                           const int32_t* hist_len, int L, uint8_t* out, int B, int HW, hipStream_t stream);

/* ---- networks (src/networks.py) -------------------------------------------------------- */

/* Conv2d(+BN folded)(+ReLU)(+residual) as one implicit-GEMM MFMA kernel: ConvBlock /
 * ResidualBlock halves / plain Conv2d (networks.py:7-35, 48-72). dtype 0 = f32, 1 = bf16.
 * in: NHWC, env b at in + b*in_env_stride (+ slot[b]*in_slot_stride when slot != NULL: gather of
 * parent latents from the node pool). w: [Cout][ks*ks*Cin] (tap-major, K-contiguous). bias f32.
 * act_bias f32 [HW][A][Cout] + act i32[B]: the dynamics net's one-hot action planes
 * (mcts.py:252-268). res: residual [B*HW][Cout] (may alias out). Cin % (dtype ? 8 : 4) == 0, Cout % 4 == 0. */
/* 1 (default): bf16 convs over >= 64K pixels with Cout % 256 == 0 (no action bias / slot gather) run on
 * a 256-pixel x 256-channel tile kernel (large images: config 3's 84x84 / 21x21); 0: always the generic one. */
int mzba_conv2d_set_variant(int v);
int mzba_conv2d(int dtype, const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                const void* w, const float* bias, const float* act_bias, const int32_t* act, int A, const void* res,
                void* out, int B, int H, int W, int Cin, int Cout, int ks, int relu, hipStream_t stream);

/* Halo-tiled 3x3 conv (bf16, config 3's large images: the 21x21 latent towers, the 42x42 / 84x84
 * representation convs; networks.py:19-35): out = act(conv3x3(in) + bias (+ res)) on contiguous NHWC images
 * of B envs, zero padding. A workgroup stages 256 consecutive output pixels plus W + 1 halo rows on each side
 * into LDS once per channel block and runs all 9 taps from it. wh = pack_lat16 of the BN-folded
 * [Cout][3][3][Cin] weights: wh[Cout/16][9*Cin/32][64][8], wh[ct][s][l][j] = W[16 ct + l % 16][32 s + 8 (l / 16) + j]
 * with the K index tap * Cin + channel. Supported: Cin 128 / 256, Cout % 256 == 0, or Cout 128 with all Cin channels
 * staged at once (the policy head's conv, networks.py:200-206; the 84x84 128-channel blocks), the staged halo within
 * the LDS (with its 16-row zero block) in one block or, at Cin 256, two 128-channel blocks (W <= 23 / 183: one
 * block at Cin 256 / 128; two blocks up to W = 183) (mzba_conv_halo_supported). Replaces
 * networks.py:19-35 ResidualBlock convs (the second with res). */
int mzba_conv_halo_supported(int H, int W, int Cin, int Cout, int ks);
/* mzba_conv_halo with a gathered input and the action planes folded into a bias table (the dynamics' first conv,
 * networks.py:117-122, 160; the same contract as mzba_conv2d's slot / act_bias arguments): env b's image at
 * in + b env_stride + slot[b] slot_stride elements (slot optional), out = act(conv3x3 + act_bias[p][act[b]][n] +
 * bias[n] (+ res)), ((acc + act_bias) + bias) in f32 as conv_igemm; act_bias [H W][A][Cout] f32 excludes res.
 * gather = 1 in the support check: a strided / gathered input or an action-bias table (Cin 256, Cout % 256 == 0,
 * one staged 256-channel block, i.e. W <= 23; 256 + 2 (W + 1) <= H W: a workgroup's staged rows within two envs). */
int mzba_conv_halo_ex_supported(int H, int W, int Cin, int Cout, int ks, int gather);
int mzba_conv_halo_ex(const void* in, long long env_stride, const int32_t* slot, long long slot_stride, const void* wh,
                      const float* bias, const float* act_bias, const int32_t* act, int A, const void* res, void* out,
                      int B, int H, int W, int Cin, int Cout, int relu, hipStream_t stream);
/* Waves per workgroup of the Cin 256 one-block halo instances: 0 default (8), 4, 8; -1 otherwise. Outputs are
 * identical for every choice (each accumulator takes its taps in the same order). */
int mzba_conv_halo_set_waves(int nw);
/* Pixels per workgroup of the Cin 256 / Cout 256 halo instances. 256-pixel form: all 256 channels staged at once
 * where the halo fits (W <= 23), else two 128-channel blocks, one workgroup per CU; 128-pixel form: two staged
 * 128-channel blocks within 80 KiB and <= 128 VGPRs, two workgroups per CU. 0 (default): the 128-pixel form where
 * the 256-pixel form stages two blocks anyway (W > 23; the same k order, the same bits); 1: the 128-pixel form
 * wherever it fits (at W <= 23 each output's taps sum block by block: bf16-rounding-level differences); 2: never;
 * -1 otherwise. */
int mzba_conv_halo_set_form(int f);
/* f32-faithful 3x3 conv on bf16 MFMAs (the f32 parity path's latent towers, networks.py:19-35): f32 NHWC in /
 * out, out = act(conv3x3(in) + bias (+ res)); every f32 operand split into three bf16 parts and each product
 * taken as the six terms down to 2^-18 (csrc/conv_x6.hip), as close to exact as an f32 conv. wx = the three
 * parts of the f32 [Cout][3][3][Cin] weights (hi = bf16(w), mid = bf16(w - hi), lo = bf16(w - hi - mid)), each
 * in mzba_conv_halo's pack_lat16 packing, back to back. Supported: Cin 128 / 256, Cout % 256 == 0, the staged
 * halo within the LDS; and the 4x5 latent at Cin 256 with Cout 256 or 128 (the pixel-tiled form, round 5: 16 envs
 * x 20 pixels per workgroup, the zero-padding taps not issued) (mzba_conv_x6_supported). */
int mzba_conv_x6_supported(int H, int W, int Cin, int Cout, int ks);
int mzba_conv_x6(const void* in, const void* wx, const float* bias, const void* res, void* out, int B, int H, int W,
                 int Cin, int Cout, int relu, hipStream_t stream);
/* mzba_conv_x6 with a gathered input and the action planes folded into a bias table (the f32 dynamics' first conv,
 * networks.py:117-122, 160; the contract of mzba_conv_halo_ex): env b's image at in + b env_stride + slot[b]
 * slot_stride elements (slot optional), out = act(conv3x3 + act_bias[p][act[b]][n] + bias[n] (+ res)),
 * ((acc + act_bias) + bias) in f32 as conv_igemm; act_bias [H W][A][Cout] f32 excludes res. gather = 1 in the
 * support check: a strided / gathered input or an action-bias table (the pixel-tiled form only: the 4x5 latent,
 * Cin 256, Cout 256 / 128). ks 3, or 1 at the 4x5 latent (the reward / value heads' 1x1 ConvBlocks, wx then the
 * three parts of [Cout][1][1][Cin]). */
int mzba_conv_x6_ex_supported(int H, int W, int Cin, int Cout, int ks, int gather);
int mzba_conv_x6_ex(const void* in, long long env_stride, const int32_t* slot, long long slot_stride, const void* wx,
                    const float* bias, const float* act_bias, const int32_t* act, int A, const void* res, void* out,
                    int B, int H, int W, int Cin, int Cout, int ks, int relu, hipStream_t stream);
/* Split-fp16 x3 form of the pixel-tiled conv (round 6; networks.py:19-35, 103-241, the reference's f32 convs):
 * every f32 operand as two fp16 parts (x = xh + xl, xh = fp16(x), xl = fp16(x - xh)) and a product as the three
 * terms xh wl + xl wh + xh wh on fp16 MFMAs with f32 accumulation — about 22 significant bits per operand, half the
 * MFMAs of the x6 form. wx3 = the two fp16 parts of w 2^k (k per output channel: max |w 2^k| in [2^14, 2^15)), each in
 * pack_lat16's packing, back to back; wscale[Cout] = 2^-k. Activations must stay below 65520 in magnitude (else the
 * output turns non-finite). Same shapes, gather and action-bias contract as mzba_conv_x6_ex at the 4x5 latent; and
 * contiguous 3x3 convs on the pre-split halo tiles (160-pixel tiles at W >= 16 for Cin 256 / 128; Cin 256, Cout % 256
 * == 0 elsewhere: the 16x20 and 8x10 representation convs) (mzba_conv_x3_supported). */
int mzba_conv_x3_supported(int H, int W, int Cin, int Cout, int ks, int gather);
int mzba_conv_x3_ex(const void* in, long long env_stride, const int32_t* slot, long long slot_stride, const void* wx3,
                    const float* wscale, const float* bias, const float* act_bias, const int32_t* act, int A,
                    const void* res, void* out, int B, int H, int W, int Cin, int Cout, int ks, int relu,
                    hipStream_t stream);
/* The x3 form's block pipeline (process-wide): 1 (default) each wave splits its own LDS-DMA rows of the next
 * 32-channel block into a second plane set during the current block's k loop (one barrier per block); 0 the
 * round-5 structure, a split phase between two barriers per block (A/B). Bit-identical. -1 on a bad value. */
int mzba_conv_x3_set_pipe(int on);
/* 2 (default): the pixel-tiled form at the 4x5 latent where its 16-env workgroups load the busiest CU less than the
 * pre-split tiles (the gathered / Cout 128 convs always), else the pre-split form where its staged rows fit (the f32
 * activations split once into bf16 hi / mid / lo planes while staging, 1.5x the f32 row; 8 waves x 32 channels),
 * else the per-read-split kernel; 3: the pixel-tiled form wherever it applies; 1: no pixel-tiled form (A/B);
 * 0: the per-read-split kernel only (A/B). The pre-split and per-read-split forms are bit-identical (same sums in
 * the same order); the pixel-tiled form sums the same products in another order (channel block, tap). */
int mzba_conv_x6_set_variant(int v);
/* Workgroup width of the pixel-tiled x6 conv (process-wide): 0 (default) 4 waves / 64 output channels where the
 * 8-wave grid (16 envs x 128 channels per workgroup) would leave CUs idle (config 2's 1 024 envs), else 8; 8 or 4
 * force it. Per 16-channel tile the arithmetic is the same, so the outputs are identical. -1 otherwise. */
int mzba_conv_x6_set_waves(int nw);
int mzba_conv_halo(const void* in, const void* wh, const float* bias, const void* res, void* out, int B, int H, int W,
                   int Cin, int Cout, int relu, hipStream_t stream);

/* Latent-resolution conv (bf16): same contract as mzba_conv2d for H*W <= 160, Cin in {64,128,256},
 * Cout % 32 == 0, but the weights are in fragment-major order wf[Cout/32][2][ks*ks][Cin/32][64][8]
 * followed by 8*64*8 padding elements (the weight ring prefetches 8 k steps past the end; see
 * DESIGN.md §conv_lat); a workgroup keeps E = 160/(H*W) envs' activations in LDS. */
int mzba_conv_lat_supported(int H, int W, int Cin, int Cout, int ks);
/* Kernel shape selection for A/B experiments (0 = default 8-wave kernel, with 3-row-tile workgroups
 * where the 5-tile grid would leave CUs idle; 1 = 4-wave 2-tile kernel; 2 = 5-row-tile workgroups only). */
int mzba_conv_lat_set_variant(int v);
/* current conv_lat variant (the learner switches to 5-row tiles for its two-stream minibatch and back) */
int mzba_conv_lat_get_variant(void);
int mzba_conv_lat(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                  const void* wf, const float* bias, const float* act_bias, const int32_t* act, int A,
                  const void* res, void* out, int B, int H, int W, int Cin, int Cout, int ks, int relu,
                  hipStream_t stream);
/* Learner (bf16, no bias fold, no ReLU): conv_lat of an NHWC batch (optionally applying the PRODUCING
 * BatchNorm while staging: pstats != NULL -> the conv input is y = [prelu](in * alpha + beta' [+ pres]),
 * alpha / beta' = pstats rows 2 / 3, and y is stored to pout, replacing mzba_bn_apply) with the consuming BatchNorm's
 * per-workgroup batch statistics computed in the epilogue (replaces bn_stats_partial /
 * bn_backward's partial pass, learn.hip). mode 1: part[chunk][Cout] = (mean, M2) of the bf16
 * outputs over the chunk's rows (-> mzba_bn_stats_final); mode 2: out = bf16(conv + res) * [y > 0]
 * (the ReLU mask of the BN output y) and part[chunk][Cout] = (sum g, sum g (x - mean)) with x the
 * BN input, mean = stats row 0 (-> mzba_bn_backward_final); mode 0: no statistics. Cout % 128 == 0;
 * res may alias out.
 * Backward prologue (pcoef != NULL): the staged input is the BN input gradient dt = ((g - (x - mean) k)
 * - mean_g) alpha of g = in and x = pres (mean, alpha = pstats rows 0, 2; mean_g, k = pcoef rows 0, 1
 * from mzba_bn_backward_coef), stored to pout (replacing mzba_bn_backward_final's apply).
 * mzba_conv_lat_bn_chunks gives the chunk count (part has nchunk * Cout float2) and rows per chunk. */
int mzba_conv_lat_bn_chunks(int B, int H, int W, int Cin, int Cout, int ks, int* nchunk, int* rpc);
int mzba_conv_lat_bn(const void* in, const void* wf, const float* bias, const void* res, void* out, int B, int H,
                     int W, int Cin, int Cout, int ks, int mode, float* part, const void* y, const void* x,
                     const float* mean, const float* pstats, const void* pres, int prelu, void* pout,
                     const float* pcoef, hipStream_t stream);
/* mzba_conv_lat_bn plus the consuming BatchNorm's finaliser in the same launch: the last workgroup of each
 * 128-channel column block (told by its add to ctr[column block]) folds every workgroup's partials (sc1 stores and
 * loads: MI355X_MICROARCH.md's hand-off table, row 1). mode 1 = mzba_bn_stats_final (fstats out [4][Cout], running
 * statistics updated when run_mean != NULL); mode 2 = mzba_bn_backward_coef (fstats in, dgamma / dbeta +=, coef out
 * [3][Cout]). The chunk statistics fold in another order than those kernels' (f32 last-place differences). ctr:
 * Cout / 128 words, zero at entry, zero again at exit, one launch in flight per word. Replaces, in the learner, the
 * BN finaliser launch after each fused conv (train_torch.py:487-528's BatchNorm2d in train mode). */
int mzba_conv_lat_bn_fin(const void* in, const void* wf, const float* bias, const void* res, void* out, int B, int H,
                         int W, int Cin, int Cout, int ks, int mode, float* part, const void* y, const void* x,
                         const float* mean, const float* pstats, const void* pres, int prelu, void* pout,
                         const float* pcoef, unsigned* ctr, float eps, float momentum, const float* gamma,
                         const float* beta, float* fstats, float* run_mean, float* run_var, float* dgamma, float* dbeta,
                         float* coef, hipStream_t stream);

/* Fused residual tower: nblocks ResidualBlock(256) on the 4x5 latent in ONE launch (networks.py:19-35,
 * 124-131, 190-197); a workgroup keeps 4 (or, for B >= 8 x CUs, 8) envs' activations in LDS for the
 * whole tower. wf16: per conv [16 col tiles][72 k steps][64 lanes][8] bf16 with taps ordered (dx, dy)
 * (agent.pack_tower_conv), convs back to back, + 8*64*8 padding elements; bias: per conv [256] f32 (BN folded). in: env b at in + b*in_env_stride
 * (+ slot[b]*in_slot_stride); out: [B][20][256] bf16. */
/* Representation-net 3x3 convs at 16x20 (networks.py:38-99, 7-35): one workgroup per (env, 10-column
 * band), 160 rows x Cout, weights in the tower packing (agent.pack_tower_conv, + 8 KB pad).
 * out = [relu](conv(in) + bias [+ res]); NHWC bf16, env strides 320*Cin / 320*Cout; out may alias res. */
int mzba_conv_band_supported(int H, int W, int Cin, int Cout, int ks);
/* band width of mzba_conv_band: 5 output columns per workgroup (default; two workgroups per CU) or 10 */
int mzba_conv_band_set_xt(int xt);
int mzba_conv_band(const void* in, const void* wf16, const float* bias, const void* res, void* out, int B, int H,
                   int W, int Cin, int Cout, int relu, hipStream_t stream);

/* ResidualBlock(C) of the representation net at 16x20 in ONE launch (networks.py:19-35, 46-92):
 * out = relu(conv2(relu(conv1(in) + b1)) + b2 + in), BN folded, both weights in the tower packing
 * (agent.pack_tower_conv, + 8 KB pad). A workgroup owns one env's 10-column band and keeps it in LDS
 * across both convs (conv1 over the band + 1 halo column each side); the outputs equal two
 * mzba_conv_band launches bit for bit. NHWC bf16; C in {128, 256}; out must not alias in. */
int mzba_conv_band_res_supported(int H, int W, int C);
int mzba_conv_band_res(const void* in, const void* w1, const float* b1, const void* w2, const float* b2, void* out,
                       int B, int H, int W, int C, hipStream_t stream);

/* Replay ingest on the device (replay_buffer.py:96-165, train_torch.py:223-225). Records of one episode
 * batch as the acting loop's sink holds them: action u8 [T][B], reward f32 [T][B], mask u8 [T][B]
 * (recorded = not prev_done, a prefix), counts i64 [T][B][3], value f32 [T][B], frame u8 [T][B][HW]
 * gray codes, frame0 u8 [B][HW] = g(s0).
 * plan: lens i32[B], rsum f32[B] (reward sums), offsets i32[B+1] = exclusive scan of the window counts
 *       (L - K + 1 for trajectories with L > min_len, else 0).
 * write: windows [j0, n) with j0 = max(0, n - cap) into ring slots (head + j) % cap: past actions
 *       i64 [cap][hist], future actions i64 [cap][K], frames u8 [cap][hist][HW], rewards / values /
 *       n-step targets f32 [cap][K], counts f32 [cap][K][3], reward sum f32 [cap]; dpow f32[T + 2]:
 *       dpow[k] = f32(discount**k) for k <= T, dpow[T + 1] = f32(discount**K) (python double pow).
 * states: out f32 [n][hist][HW] = lut8[code & 7] for ring slots slots[n] (the learner's input). */
int mzba_replay_plan(const uint8_t* action, const float* reward, const uint8_t* mask, const int64_t* counts,
                     const float* value, const uint8_t* frame, const uint8_t* frame0, int T, int B, int HW, int K,
                     int min_len, int32_t* lens, float* rsum, int32_t* offsets, hipStream_t stream);
int mzba_replay_write(const uint8_t* action, const float* reward, const uint8_t* mask, const int64_t* counts,
                      const float* value, const uint8_t* frame, const uint8_t* frame0, int T, int B, int HW,
                      const int32_t* lens, const float* rsum, const int32_t* offsets, int n_windows,
                      int64_t* past_actions, int64_t* future_actions, uint8_t* states, float* rewards,
                      float* counts_out, float* values_out, float* targets, float* reward_sum, int cap, int head,
                      int K, int hist, const float* dpow, hipStream_t stream);
int mzba_replay_states(const uint8_t* states, const int32_t* slots, int n, const float* lut8, float* out, int hist,
                       int HW, hipStream_t stream);

/* kernel choice for experiments/tests: 0 by batch (default), 1 four-env 8-wave kernel, 2 eight-env
 * kernel, 3 four-env 4-wave kernel */
int mzba_tower_set_variant(int v);
/* kernel mzba_tower runs for batch B: 3 four-env 4-wave (workgroup = 4 envs, 4 waves of 64 output channels)
 * below 8 x CUs envs, else 2 eight-env (workgroup = 8 envs, 4 waves: half the weight stream per env);
 * 1 = the four-env 8-wave kernel (32 channels per wave; by variant only). All take agent.pack_tower_conv
 * weights. The 4-wave kernels stage the tower biases in LDS: nblocks <= 24 (else -5). */
int mzba_tower_plan(int B);
/* device scratch bytes mzba_tower needs for batch B (0 for both kernels; the ws argument may be null) */
long long mzba_tower_ws_bytes(int B);
int mzba_tower(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride, void* out,
               const void* wf16, const float* bias, int nblocks, int B, void* ws, long long ws_bytes,
               hipStream_t stream);
/* Fused per-simulation nets around the tower (every plan): the dynamics ConvBlock
 * before it and the reward / policy / value heads after it run in the same launch, so one
 * dynamics step and one prediction step are one kernel each (networks.py:151-167, 200-241,
 * 314-328; utils.py:74-81). */
/* One simulation's tree update folded into the fused prediction step: after the heads, each env's
 * thread backs up this simulation's leaf (mcts.py:203-234) and, when sim + 1 < S, selects the next
 * leaf (mcts.py:136-182). Fields as the mzba_mcts_* tree arguments. */
typedef struct mzba_tree_step {
  void* nodes;
  float* root_sum;
  uint32_t* calls;
  int32_t* leaf_parent;
  int32_t* leaf_action;
  int32_t* depth;
  int32_t* path;
  const float* sqrt_tab;
  const float* c_tab;
  int B, S, env_offset, search_id;
  uint64_t seed;
  const int32_t* ctx;
  int sim;
  float gamma;
  const float* r;         /* decoded rewards of this simulation's dynamics step [B] */
} mzba_tree_step;

/* Pixel-tiled tower (csrc/towerp.hip): the same math as mzba_tower on 16 envs per workgroup with one
 * 16-row MFMA tile per latent pixel (no padding taps issued); same weight packing and I/O layout. */
typedef struct mzba_tower_ext {
  /* prologue: dynamics ConvBlock 259->256 = 3x3 conv (tower packing) + bias + per-(position,
   * action) bias table [20][A][256] f32 (the action planes folded in), ReLU; w0 = NULL: none */
  const void* w0;
  const float* b0;
  const float* act_bias;
  const int32_t* act;
  int A;
  /* epilogue: 0 none (out = tower output); 1 dynamics: reward ConvBlock1x1 256->256 (we1/be1) +
   * Linear lw[0] -> lO[0] logits -> decode to dec[0][B], then the per-env min-max scaled latent
   * to out (may be NULL when pool is set: the node-pool slot is the only copy, as in the search) and
   * to pool slot pool_slot; 2 prediction: policy ConvBlock3x3 256->128 (we3/be3) and
   * value ConvBlock1x1 256->128 (we1/be1), Linear lw[0] -> softmax dec[0][B][lO[0]],
   * Linear lw[1] -> decode dec[1][B] */
  int epilogue;
  const void* we3;
  const float* be3;
  const void* we1;
  const float* be1;
  const void* lw[2];      /* bf16 [16][20*C], (position, channel) order, rows >= lO zero */
  const float* lb[2];
  int lO[2];
  float* logits[2];       /* optional [B][lO] */
  float* dec[2];
  void* pool;             /* bf16 latent node pool (epilogue 1), may be NULL */
  long long pool_env_stride;
  int pool_slot;
  float smin, smax;       /* support range */
  const mzba_tree_step* tree;  /* epilogue 2 only, may be NULL */
  int elem;                    /* LDS image / weight element type: 0 bf16, 1 fp16 (weights w0, we1, we3, lw and
                                  the tower packs in fp16; latents in / out stay bf16) */
  int plan;                    /* tower kernel: 0 = mzba_tower_plan(B) at launch; 1 / 2 / 3 / 4 = that kernel (the
                                  runner records the plan it packed for and launches exactly that one) */
} mzba_tower_ext;
int mzba_tower_fused(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                     void* out, const void* wf16, const float* bias, int nblocks, int B,
                     const mzba_tower_ext* ext, hipStream_t stream);

/* Pixel-tiled tower kernel (csrc/towerp.hip; plan 4 of mzba_tower / mzba_tower_fused): 16 envs per
 * workgroup, one 16-row MFMA tile per latent pixel, so the 3x3 taps that fall on the 4x5 latent's
 * zero padding are never issued; bit-identical to plans 2/3 on the same weight packing and I/O
 * layout. mzba_towerp_fused takes mzba_tower_fused's arguments (bf16, or ext->elem == 1: the fp16 dynamics net);
 * mzba_towerp is the plain tower (mzba_tower's arguments without the workspace). */
int mzba_towerp_fused(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride,
                      void* out, const void* wf16, const float* bias, int nblocks, int B,
                      const mzba_tower_ext* ext, hipStream_t stream);
int mzba_towerp(const void* in, long long in_env_stride, const int32_t* slot, long long in_slot_stride, void* out,
                const void* wf16, const float* bias, int nblocks, int B, hipStream_t stream);

/* Representation tail in one launch (networks.py:86-99, 271-280, 314-328): AvgPool2d of the 16x20
 * activations after the last full-resolution block (in [B][320][256] bf16), nblocks ResidualBlock(256)
 * at 8x10 (wf16: their 2 nblocks convs BN-folded in the tower packing, back to back + 8 KB pad; bias
 * [2 nblocks][256] f32), AvgPool2d to 4x5, _scale_state; the root latent to out [B][20][256] bf16 and,
 * when pool != NULL, to pool + b * pool_env_stride. nblocks <= 24. */
int mzba_rep_tail(const void* in, void* out, void* pool, long long pool_env_stride, const void* wf16,
                  const float* bias, int nblocks, int B, hipStream_t stream);

/* nblocks ResidualBlock(256) at 16x20 in one launch (networks.py:73-82; csrc/repblocks.hip): one env per
 * workgroup, its whole 16x20x256 image LDS-resident across the blocks; mzba_conv_band_res's tap order per
 * accumulator, with bias + residual added first (equal to the band path within f32 rounding).
 * in / out [B][320][256] bf16 NHWC (distinct), wf16 the 2 nblocks convs BN-folded in the tower packing
 * back to back (+ 8 KB pad), bias [2 nblocks][256] f32. nblocks <= 24. */
int mzba_rep_blocks(const void* in, void* out, const void* wf16, const float* bias, int nblocks, int B,
                    hipStream_t stream);

/* The representation trunk at 16x20 in one launch (RepresentationNetwork, networks.py:46-82: Conv2d
 * 2L -> c0, n0 ResidualBlock(c0), Conv2d c0 -> c1, n1 ResidualBlock(c1); everything before the first
 * AvgPool2d; csrc/repblocks.hip): one env per workgroup, its image LDS-resident throughout, replacing the
 * band launches and mzba_rep_blocks. 2L = 64, c0 = 128, c1 = 256. in [B][320][64] bf16 NHWC (the
 * representation input), out [B][320][256] bf16 NHWC (distinct). w / b: HOST arrays of the
 * 2 n0 + 2 + 2 n1 convs' device pointers in network order (stem, each c0 block's conv1 / conv2, widening
 * conv, each c1 block's conv1 / conv2): weights in the tower packing (the last followed by 8 KB of
 * padding), biases [Cout] f32 (BN folded into the block convs). 2 n0 + 2 + 2 n1 <= 56. */
int mzba_rep_trunk(const void* in, void* out, const void* const* w, const float* const* b, int n0, int n1, int B,
                   hipStream_t stream);

/* nn.AvgPool2d(2, 2) (networks.py:44), NHWC. */
int mzba_avgpool2(int dtype, const void* in, void* out, int B, int H, int W, int C, hipStream_t stream);

/* MuZeroAgent._scale_state (networks.py:314-328): per-env min-max over n values; writes out and,
 * when pool != NULL, pool + b*pool_env_stride + (slot_arr ? slot_arr[b] : slot_const)*slot_stride. */
int mzba_scale_state(int dtype, const void* h, void* out, void* pool, long long pool_env_stride,
                     const int32_t* slot_arr, int slot_const, long long slot_stride, int B, int n,
                     hipStream_t stream);

/* Linear heads (networks.py:147-148, 207-208, 221-222) + decode: dec 0 = softmax (mcts.py:100,199),
 * dec 1 = ScalarTransforms.inverted_softmax_expectation (utils.py:74-81). w: [O][K] f32 in NHWC
 * flatten order; logits optional. */
int mzba_heads(int dtype, int nheads, const void* x0, const float* w0, const float* b0, int K0, int O0, int dec0,
               float* logits0, float* out0, const void* x1, const float* w1, const float* b1, int K1, int O1,
               int dec1, float* logits1, float* out1, float smin, float smax, int B, hipStream_t stream);
/* f32 heads: 1 (default) the f32-MFMA form (16 envs per workgroup; K % 16 == 0), 0 the per-thread FMA form (A/B). */
int mzba_heads_set_variant(int v);

/* ScalarTransforms.inverted_softmax_expectation (utils.py:74-81) on rows x n f32 logits. */
int mzba_support_decode(const float* logits, float* out, int rows, int n, float smin, float smax, hipStream_t stream);

/* bf16 path of mzba_heads as a small MFMA GEMM (16 envs per workgroup): x* [B][K] bf16, w* [16][K]
 * bf16 with zero rows >= O, K % 32 == 0. */
int mzba_heads_bf16(int nheads, const void* x0, const void* w0, const float* b0, int K0, int O0, int dec0,
                    float* logits0, float* out0, const void* x1, const void* w1, const float* b1, int K1, int O1,
                    int dec1, float* logits1, float* out1, float smin, float smax, int B, hipStream_t stream);

/* ---- latent MCTS (src/mcts.py:MCTSSearchVec) ------------------------------------------- */
/* Every tree entry point takes an optional device step context ctx (int32[3]: search id, step
 * index, episode row); when non-NULL its ctx[0] replaces search_id, so one captured HIP graph
 * replays every search. Tree buffers (device): nodes [B][S+1] x mzba_mcts_node_bytes(), root_sum f32[B], calls u32[B],
 * leaf_parent/leaf_action/depth i32[B], path i32[B][S+1]; sqrt_tab/c_tab f32[S+1] =
 * f32(sqrt(n)), f32(c1 + log((n+c2+1)/c2)) computed in double on the host (mcts.py:285-289). */
int mzba_mcts_node_bytes(void);

/* _initialize_trees + _expand_root_nodes (mcts.py:73-134): root P = f32(w_pol*pi) + f32(w_noise*noise),
 * noise = noise_in or Dirichlet(alpha) from Philox stream 2 (written to noise_out), first ucb_action.
 * w_dev (optional, device f32[2]) replaces (w_pol, w_noise): the train loop's noise_weight schedule
 * (train_torch.py:134-135) then needs no new graph capture. */
int mzba_mcts_root(void* nodes, float* root_sum, uint32_t* calls, int32_t* leaf_parent, int32_t* leaf_action,
                   int32_t* depth, int32_t* path, const float* sqrt_tab, const float* c_tab, int B, int S,
                   int env_offset, int search_id, uint64_t seed, const int32_t* ctx, const float* v_root, const float* pi_root,
                   const float* noise_in, float* noise_out, float w_pol, float w_noise, const float* w_dev, float alpha,
                   hipStream_t stream);

/* _select_nodes (mcts.py:136-182) for simulation sim >= 1 (ucb_action :281-298). */
int mzba_mcts_select(void* nodes, float* root_sum, uint32_t* calls, int32_t* leaf_parent, int32_t* leaf_action,
                     int32_t* depth, int32_t* path, const float* sqrt_tab, const float* c_tab, int B, int S,
                     int env_offset, int search_id, uint64_t seed, const int32_t* ctx, int sim, hipStream_t stream);

/* _backup (mcts.py:203-234) with decoded r[B], v[B], pi[B][3] of the expanded leaves. */
int mzba_mcts_backup(void* nodes, float* root_sum, uint32_t* calls, int32_t* leaf_parent, int32_t* leaf_action,
                     int32_t* depth, int32_t* path, const float* sqrt_tab, const float* c_tab, int B, int S,
                     int env_offset, int search_id, uint64_t seed, const int32_t* ctx, int sim, const float* r, const float* v,
                     const float* pi, float gamma, hipStream_t stream);

/* _compute_results (mcts.py:236-250): counts i64[B][3], values f32[B] = f32(double(root_sum)/S). */
int mzba_mcts_results(void* nodes, float* root_sum, uint32_t* calls, int32_t* leaf_parent, int32_t* leaf_action,
                      int32_t* depth, int32_t* path, const float* sqrt_tab, const float* c_tab, int B, int S,
                      int env_offset, int search_id, uint64_t seed, const int32_t* ctx, int64_t* counts, float* values,
                      hipStream_t stream);

/* Temperature sampling (train_torch.py:191-198 `visit_counts ** (1/self.temperature)` / sum(dim=1) then
 * Categorical(probs[i]).sample()): probs bit-identical to torch's CPU evaluation on the reference's whole
 * (n_envs_total, 3) int64 batch tensor (csrc/torch_pow.h: SLEEF powf_u10 on the vectorized part, f32(pow(double))
 * on the scalar tails; vec_block = 32 for the AVX512 host the fixtures came from, 16 for AVX2; pow_threads =
 * the reference process's intra-op threads: from 32768 elements on, torch splits the tensor into per-thread
 * chunks, each with its own scalar tail), then the inverse CDF of u = Philox uniform(env + env_offset,
 * stream 3, step, 0). inv_t = 1/T in double (Python's `1/self.temperature`); inv_t_dev (optional,
 * device f64[1]) overrides it (graph-replayable temperature schedule). probs_out (optional) f32[B][3]. */
int mzba_sample_actions(const int64_t* counts, int64_t* action, float* probs_out, int B, double inv_t,
                        const double* inv_t_dev, int n_envs_total, int vec_block, int pow_threads, int env_offset,
                        int step, uint64_t seed, const int32_t* ctx, hipStream_t stream);

/* torch's CPU `int64 counts ** e` (the power of mzba_sample_actions) for n elements at flat positions
 * [start, start + n) of a tensor of n_total elements: out f32[n]. Exposed for the parity tests. */
int mzba_torch_pow(const int64_t* counts, float* out, long long n, double e, long long start, long long n_total,
                   int vec_block, int pow_threads, hipStream_t stream);

/* Trajectory-sink row of the search results: rec_counts[t][b] = counts[b], rec_values[t][b] = values[b],
 * t = ctx ? ctx[2] : t (replay_buffer.py:17-35 visit_counts / values). */
int mzba_record_results(const int64_t* counts, const float* values, int64_t* rec_counts, float* rec_values, int B,
                        int t, const int32_t* ctx, hipStream_t stream);

/* ctx[0..2] += 1 (end of one captured acting step). */
int mzba_ctx_advance(int32_t* ctx, hipStream_t stream);

/* ===================== learner: one minibatch of RLSystem._training_stage
 * (train_torch.py:380-407) — _k_step_rollout (:487-528) with train-mode BN, loss_fn (:33-66),
 * backward, torch.optim.Adam(lr, weight_decay=1e-4) (networks.py:268). NHWC activations, dtype
 * 0 = f32, 1 = bf16 storage; statistics, gradients and parameters f32. ws = caller scratch. */

/* BatchNorm2d forward statistics in train mode (nn.BatchNorm2d in ConvBlock / ResidualBlock,
 * networks.py:7-35): stats[4][C] = (mean, invstd, gamma*invstd, beta - mean*gamma*invstd) over the
 * M rows of x [M][C]; running_mean / running_var (may be NULL) updated with momentum and the
 * unbiased variance. C % 4 == 0; ws >= ceil(M/64)*C*8 bytes. */
int mzba_bn_stats(int dtype, const void* x, int M, int C, float eps, float momentum, const float* gamma,
                  const float* beta, float* stats, float* run_mean, float* run_var, void* ws, long long ws_bytes,
                  hipStream_t stream);
/* out = x*stats[2] + stats[3] (+ res) (ReLU if relu); out may alias x or res. C % 4 == 0. */
int mzba_bn_apply(int dtype, const void* x, const float* stats, const void* res, int relu, void* out, int M, int C,
                  hipStream_t stream);
/* BN (+ReLU) backward: if y != NULL, dy *= [y > 0] in place (the ReLU after the BN / residual
 * add); dgamma += sum(dy*xhat), dbeta += sum(dy); dx = (dy - (x-mean)*k - mean(dy))*gamma*invstd.
 * C % 4 == 0; ws >= ceil(M/64)*C*8 + 12*C bytes. */
int mzba_bn_backward(int dtype, void* dy, const void* y, const void* x, const float* stats, int M, int C,
                     float* dgamma, float* dbeta, void* dx, void* ws, long long ws_bytes, hipStream_t stream);
/* The final passes of mzba_bn_stats / mzba_bn_backward from per-chunk partials computed elsewhere
 * (mzba_conv_lat_bn): chunk k covers rows [k*rpc, min(M, (k+1)*rpc)). backward: g is already
 * ReLU-masked; ws >= 12*C bytes. */
int mzba_bn_stats_final(const float* part, int nchunk, int rpc, int M, int C, float eps, float momentum,
                        const float* gamma, const float* beta, float* stats, float* run_mean, float* run_var,
                        hipStream_t stream);
int mzba_bn_backward_final(int dtype, const void* g, const void* x, const float* stats, const float* part, int nchunk,
                           int M, int C, float* dgamma, float* dbeta, void* dx, void* ws, long long ws_bytes,
                           hipStream_t stream);
/* mzba_bn_backward_final split in two: coef (dgamma / dbeta += and coef[3][C] = (mean_g, k,
 * gamma*invstd)) and apply (dx = ((g - (x - mean) k) - mean_g) gamma invstd). */
int mzba_bn_backward_apply(int dtype, const void* g, const void* x, const float* stats, const float* coef, void* dx,
                           int M, int C, hipStream_t stream);
int mzba_bn_backward_coef(const float* part, int nchunk, int M, int C, const float* stats, float* dgamma, float* dbeta,
                          float* coef, hipStream_t stream);
/* Weight packs from the f32 master weights w [Cout][taps][Cin]: flip = 0: cast copy (forward);
 * flip = 1: wt [cin_used][taps][Cout] = w[co][taps-1-tap][ci] (the input-gradient convolution). */
int mzba_conv_wpack(int dtype, const float* w, void* wt, int Cout, int taps, int Cin, int cin_used, int flip,
                    hipStream_t stream);
/* bf16 packs for mzba_conv_lat (layout 1) / mzba_conv_band (layout 2, 3x3) from the f32 master
 * weights w [Cout][taps][Cin]: logical W'[n][tap][c] = flip ? w[c][taps-1-tap][n] : w[n][tap][c]
 * (N x Cc; flip: N <= Cin, Cc = Cout), + pad zero elements. */
int mzba_conv_pack_bf16(const float* w, void* out, int Cout, int taps, int Cin, int N, int Cc, int flip, int layout,
                        long long pad, hipStream_t stream);
/* njobs mzba_conv_pack_bf16 calls in ceil(njobs / 32) launches (the learner's per-minibatch packs, round 5):
 * w[j], out[j] (16-B aligned), prm[8 j .. 8 j + 7] = {Cout, taps, Cin, N, Cc, flip, layout, pad} (pad % 8 == 0);
 * host arrays; the same outputs as the separate calls. */
int mzba_conv_pack_bf16_multi(const float* const* w, void* const* out, const int* prm, int njobs, hipStream_t stream);
/* Conv2d weight / bias gradient: dw [Cout][ks*ks][Cin] += sum_m dy[m][co] * x_tap[m][ci],
 * db [Cout] += sum_m dy[m][co] (db may be NULL). x NHWC [B][H][W][Cin], dy [B][H][W][Cout]. */
long long mzba_conv_wgrad_ws_bytes(int B, int H, int W, int Cin, int Cout, int ks);
/* bf16 3x3 weight-gradient kernel choice: 1 (default) whole zero-bordered images per tile, all 9 taps;
 * 0 one tap per tile (the kernel used for 1x1 and f32). */
int mzba_conv_wgrad_set_variant(int v);
/* the whole-image kernel's form (per host thread): 2 (default) pixel rows with 64-co wave tiles — k over the
 * real pixels of a stage, out-of-image taps read a zero row (round 6); 1 the same with 32-co wave tiles
 * (bit-identical to 2, more LDS fragment reads); 3 form 2 with software-pipelined k steps (bit-identical,
 * measured slower, A/B); 0 zero-bordered images (round 5, A/B; the same sums in a different f32 order); -1 for
 * another value. */
int mzba_conv_wgrad_set_form(int v);
int mzba_conv_wgrad(int dtype, const void* x, const void* dy, int B, int H, int W, int Cin, int Cout, int ks,
                    float* dw, float* db, void* ws, long long ws_bytes, hipStream_t stream);
/* The same over nseg (<= 8) (x, dY) segments of B envs each, reduced in one contraction (the K
 * unrolled uses of one weight; ws sized by mzba_conv_wgrad_ws_bytes(nseg * B, ...)). xs / dys:
 * host arrays of device pointers. */
int mzba_conv_wgrad_segs(int dtype, const void* const* xs, const void* const* dys, int nseg, int B, int H, int W,
                         int Cin, int Cout, int ks, float* dw, float* db, void* ws, long long ws_bytes,
                         hipStream_t stream);
/* nn.AvgPool2d(2, 2) backward: dx [B][H][W][C] = dy[y/2][x/2] / 4. */
int mzba_avgpool2_backward(int dtype, const void* dy, void* dx, int B, int H, int W, int C, hipStream_t stream);
/* y += x (n elements). */
int mzba_axpy(int dtype, void* y, const void* x, long long n, hipStream_t stream);
/* _scale_state forward (networks.py:314-328) recording minmax[B][2] and the NHWC index of the first
 * min / max in NCHW flatten order (torch.min/max(dim=1) index semantics) in argminmax[B][2]. */
int mzba_scale_forward(int dtype, const void* h, void* out, float* minmax, int32_t* argminmax, int B, int HW, int C,
                       hipStream_t stream);
/* _scale_state backward: dh (= or +=) autograd of (h - min)/(max - min + 1e-8), min / max gradients
 * routed to the recorded indices. */
int mzba_scale_backward(int dtype, const void* dy, const void* h, const float* minmax, const int32_t* argminmax,
                        void* dh, int B, int n, int accumulate, hipStream_t stream);
/* nn.Linear heads (networks.py:147, 207, 221) on an NHWC image: out[b][o] = bias[o] + sum_k w[o][k] x[b][k],
 * k = pixel*C + channel (the reference's (c, y, x) flatten order is permuted into the weight layout). */
int mzba_linear_forward(int dtype, const void* x, const float* w, const float* bias, float* out, int B, int K, int O,
                        hipStream_t stream);
long long mzba_linear_ws_bytes(int B, int K, int O);
/* dx (= or += when accumulate; NULL = skip) = dy w; dw += dy^T x; db += sum_b dy. */
int mzba_linear_backward(int dtype, const void* x, const float* w, const float* dy, void* dx, int accumulate,
                         float* dw, float* db, int B, int K, int O, void* ws, long long ws_bytes, hipStream_t stream);
/* loss_fn (train_torch.py:33-66) over logits [K][B][ns|na] with targets from replay rows slots[b]
 * (slots NULL: row b) of rewards [.][K], targets [.][K], counts [.][K][na]: supports_representation
 * (utils.py:30-64) two-hot targets, KL(batchmean) x3, loss[4] = (total, reward, value, policy) and the
 * logit gradients of the total. */
int mzba_learner_loss(const float* logit_r, const float* logit_v, const float* logit_p, const float* rewards,
                      const float* targets, const float* counts, const int32_t* slots, int B, int K, int ns, int na,
                      float smin, float smax, float* dlogit_r, float* dlogit_v, float* dlogit_p, float* loss,
                      hipStream_t stream);
/* The same outputs, bit for bit, over many workgroups (a thread per (window, step) row, then one reduction
 * workgroup folding the rows in mzba_learner_loss's order): ws >= mzba_learner_loss_ws_bytes(B, K) bytes. */
long long mzba_learner_loss_ws_bytes(int B, int K);
int mzba_learner_loss_ws(const float* logit_r, const float* logit_v, const float* logit_p, const float* rewards,
                         const float* targets, const float* counts, const int32_t* slots, int B, int K, int ns, int na,
                         float smin, float smax, float* dlogit_r, float* dlogit_v, float* dlogit_p, float* loss,
                         void* ws, long long ws_bytes, hipStream_t stream);
/* Adam with L2 weight decay, torch single-tensor order: g = grad + wd*p; m += (1-b1)(g - m);
 * v = v*b2 + (1-b2)*g*g; p += (-step_size*m) / (sqrt(v)/bc2_sqrt + eps). Host computes
 * neg_step = -lr/(1-b1^t), bc2_sqrt = sqrt(1-b2^t) in double (python float semantics). */
int mzba_adam(float* p, const float* grad, float* m, float* v, long long n, float neg_step, float one_m_b1, float b2,
              float one_m_b2, float bc2_sqrt, float eps, float weight_decay, hipStream_t stream);
/* The same with the scalars in device memory: scalars = {neg_step, 1-b1, b2, 1-b2, bc2_sqrt, eps,
 * weight_decay} (f32[7]), so a captured minibatch graph replays with per-step bias corrections. */
int mzba_adam_dev(float* p, const float* grad, float* m, float* v, long long n, const float* scalars,
                  hipStream_t stream);
/* Representation input of a minibatch (_prepare_minibatch + _encode_actions, train_torch.py:437-470,
 * 279-293) straight from the replay ring: out [B][HW][Cp] = (lut[frame code] x L, a/3 x L, 0...). */
int mzba_learner_input(int dtype, const uint8_t* states, const int64_t* past_actions, const int32_t* slots,
                       const float* lut8, void* out, int B, int L, int HW, int Cp, hipStream_t stream);
/* Dynamics input (_encode_action_dynamics, train_torch.py:295-311): out [B][HW][Cp] =
 * (h [B][HW][C], one-hot(future_actions[slots[b]][k]) x A, 0...). */
int mzba_dyn_input(int dtype, const void* h, const int64_t* future_actions, const int32_t* slots, int K, int k,
                   void* out, int B, int HW, int C, int A, int Cp, hipStream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* MZBA_H */
