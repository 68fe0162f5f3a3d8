/*
 * cbev.h — C-ABI of the MI355X batched CarlaBEV step (libcbev.so).
 *
 * The reference has no FFI: its "operator API" for this path is the Gymnasium
 * surface of `CarlaBEV.envs.carlabev.CarlaBEV` wrapped by `make_env`
 * (`CarlaBEV/envs/__init__.py:108-120`, a `SyncVectorEnv`). Each entry point
 * below replaces the per-env Python call chain named next to it, batched over
 * N environments whose state lives in device memory as fixed-size records
 * (include/cbev_layout.h). The Python facade (carlabev_env_amd/vector_env.py)
 * binds these symbols with ctypes; INTEGRATION.md shows the binding.
 *
 * Conventions: every buffer argument is a plain device pointer (HBM) unless
 * named *_host; sizes are element counts; `stream` is a hipStream_t passed as
 * void* (NULL = default stream). All launches are asynchronous on `stream`.
 * Functions return 0 on success and a negative code on error; the message is
 * available from cbev_last_error() (thread-local). Calls on one context are
 * not re-entrant.
 */
#ifndef CBEV_H
#define CBEV_H

#include <stdint.h>

#include "cbev_layout.h"

#ifdef __cplusplus
extern "C" {
#endif

#define CBEV_ABI_VERSION 7

typedef struct cbev_ctx cbev_ctx;

/* error codes */
enum { CBEV_OK = 0, CBEV_EINVAL = -1, CBEV_EHIP = -2, CBEV_ESTATE = -3 };

int cbev_abi_version(void);
int cbev_params_size(void);                         /* sizeof(cbev_params) */
int cbev_layout_of(const cbev_caps* caps, cbev_layout* out);
/* comma-separated field names of a record group: 0 HD, 1 HI, 2 AD, 3 AI, 4 TI */
const char* cbev_field_names(int group);
const char* cbev_last_error(void);

/* Context = the static world of `CarlaBEV._setup` (carlabev.py:56-72):
 * renderer geometry, action table, reward parameters, record capacities.
 * Replaces `BaseMap.__init__` (world.py:33-67) + `build_reward_fn`. */
int cbev_create(const cbev_params* params, const cbev_caps* caps, int device, cbev_ctx** out);
void cbev_destroy(cbev_ctx* ctx);

/* Upload the padded class map (render surface of world.py:_build_padded_render_map,
 * one palette id per texel, render_h rows of map_pitch bytes). Host pointer,
 * copied into context-owned HBM. Replaces load_map (envs/utils.py:49-62). */
int cbev_set_map(cbev_ctx* ctx, const uint8_t* padded_map_host, int64_t bytes);

/* One `CarlaBEV.step(action)` (carlabev.py:223-231) for n envs: k_actors (when
 * the record has actor slots), k_ego (ego update + collision / reward /
 * termination), k_raster (the observation), in that order on `stream`:
 *   records      n state records (record_bytes each), updated in place
 *   actions      int32[n] discrete indices, or float32[n][3] continuous
 *   frames       uint8[n][S][S] palette-id observation (render(), carlabev.py:233-249)
 *   reward       float64[n]; term, trunc uint8[n]; cause int32[n] (CBEV_CAUSE_*)
 *   info         float32[n][CBEV_INFO_FLOATS] per-step comfort/control export or NULL */
#define CBEV_INFO_FLOATS 16
int cbev_step(cbev_ctx* ctx, void* records, int n, const void* actions, uint8_t* frames, double* reward,
              uint8_t* term, uint8_t* trunc, int32_t* cause, float* info, void* stream);

/* Episode statistics on the device (Stats, src/deeprl/stats.py:87-148, and
 * CarlaBEV._check_termination, carlabev.py:177-185), so `infos["episode_info"]`
 * needs no per-step host work. The caller owns the buffers (device memory):
 *   stats   cbev_episode_stats[n], zeroed before first use, kept across episodes
 *   rows    float64[ring][n][CBEV_EP_COUNT]; counts int32[ring], zeroed
 * Step s (the s-th cbev_step after this call, from 0) writes one row per env
 * that terminated into rows[s % ring] (in no particular order, counts[s % ring]
 * of them) and zeroes counts[(s + 1) % ring], so a slot stays readable until
 * step s + ring - 1 is queued (ring >= 3). cbev_reset / cbev_reset_frames stamp
 * each reset env's episode start on the device clock (CBEV_EP_SECONDS).
 * stats = NULL turns it off. Not stream-ordered: call it between steps. A slot
 * holds at most n rows: a step replayed from a graph (which zeroes the same next
 * slot every replay) keeps counting in counts[] but writes no row past them. */
int cbev_set_episode_stats(cbev_ctx* ctx, void* stats, int n, double* rows, int32_t* counts, int ring);
/* Slot of the latest step's rows (-1 when off) and the step count. */
int cbev_episode_slot(const cbev_ctx* ctx, int64_t* step_count);
/* Rate of the device clock the episode times use. */
int cbev_wall_clock_hz(const cbev_ctx* ctx, double* hz);

/* Episodes terminated in all cbev_step calls since cbev_create (synchronises):
 * the reset demand a host scene feed has to meet. */
int cbev_termination_count(cbev_ctx* ctx, int64_t* count);

/* Errors the kernels detect are not stream-ordered return codes: they set bits
 * of a context error word, read (and cleared, if clear != 0) by this call,
 * which synchronises the device.
 *   CBEV_ERR_ACTION_INDEX  a discrete action outside [-n, n) (the reference's
 *                          IndexError in discrete_actions[int(action)],
 *                          envs/spaces.py:46); that env stepped action 0.
 *                          Negative indices in [-n, 0) count from the end. */
#define CBEV_ERR_ACTION_INDEX 1
/*   CBEV_ERR_RASTER_WINDOW a raster tile's crop window exceeded its LDS bound
 *                          (an internal invariant; the frame is not valid). */
#define CBEV_ERR_RASTER_WINDOW 2
/*   CBEV_ERR_RETREAT_ROUTE a StopReturn retreat would rebuild a route of more
 *                          than 64 points in a context of at most 64 actor
 *                          slots (scene packing refuses such actors; that actor
 *                          keeps its route) */
#define CBEV_ERR_RETREAT_ROUTE 4
int cbev_error_flags(cbev_ctx* ctx, int32_t* flags_host, int clear);

/* Reset the envs selected by mask (uint8[n], NULL = all):
 *   if bank != NULL: records[i] = bank[b] with b = bank_idx[i], or, when
 *   bank_idx == NULL, b = (i + bank_offset) % n_bank (device-side scene bank);
 *   then render the reset observation (BaseMap.reset: theta = 0, no actors,
 *   world.py:92-100) into every slot of frames = uint8[n_frames][n][S][S]
 *   (the frame-stack ring: FrameStackObservation pads with the reset frame;
 *   n_frames = 1 for a plain frame buffer).
 * Replaces `CarlaBEV.reset` after scene generation (carlabev.py:96-148) and the
 * wrappers' reset path. One launch. */
int cbev_reset(cbev_ctx* ctx, void* records, int n, const void* bank, int n_bank, const uint8_t* mask,
               const int32_t* bank_idx, int bank_offset, uint8_t* frames, int n_frames, void* stream);

/* Reset observations of a static scene bank, rendered once: frames = uint8[n_bank][S][S],
 * frames[b] = the observation cbev_reset would render for bank[b] (BaseMap.reset draws
 * no actors, world.py:92-100, so it depends on the bank record only). */
int cbev_bank_frames(cbev_ctx* ctx, const void* bank, int n_bank, uint8_t* frames, void* stream);

/* cbev_reset from a bank whose reset observations were rendered by cbev_bank_frames:
 * the same records and ring contents as cbev_reset(ctx, records, n, bank, n_bank, mask,
 * bank_idx, bank_offset, frames, n_frames, stream), by copies only. */
int cbev_reset_frames(cbev_ctx* ctx, void* records, int n, const void* bank, int n_bank, const uint8_t* mask,
                      const int32_t* bank_idx, int bank_offset, const uint8_t* bank_frames, uint8_t* frames,
                      int n_frames, void* stream);

/* `reset(options={"reset_mask": mask})` (SyncVectorEnv.reset -> CarlaBEV.reset,
 * carlabev.py:96-148) from a bank with cached reset frames, each reset after a
 * termination a fresh bank row: every env with mask[e] != 0 (uint8[n], read
 * when the launch runs) takes bank row (e + j * cbev_bank_stride(n_bank)) %
 * n_bank, j = the env's terminations so far (counted by cbev_step on the device
 * from 0 at cbev_create; the stride is coprime with n_bank, so each env walks
 * the whole bank before a scene repeats for it; a reset with no termination
 * since the last one takes the same row again). The row of an env depends on
 * that env alone and no reset writes the counts (ABI 7; before, a global cursor
 * dealt rows in env-id order, which made every workgroup of the folded reset
 * read the whole mask). Records and ring contents as cbev_reset_frames with
 * those bank rows. One launch, no host sync; n <= 2^20. */
int cbev_reset_masked(cbev_ctx* ctx, void* records, int n, const uint8_t* mask, const void* bank, int n_bank,
                      const uint8_t* bank_frames, uint8_t* frames, int n_frames, void* stream);
/* The canonical loop's reset, `reset(options={"reset_mask": terminated})`
 * (tools/debug_env.py:56-132): cbev_reset_masked with mask = the `term` buffer
 * of the last cbev_step on this context (n must be that step's n). */
int cbev_reset_terminated(cbev_ctx* ctx, void* records, int n, const void* bank, int n_bank,
                          const uint8_t* bank_frames, uint8_t* frames, int n_frames, void* stream);
/* The sum of the per-env termination counts (synchronises the device): the
 * bank rows the canonical loop's resets have handed out since cbev_create. */
int cbev_bank_cursor(cbev_ctx* ctx, int64_t* cursor);
/* The per-env termination counts j of envs 0 .. n-1 (synchronises). */
int cbev_reset_counts(cbev_ctx* ctx, uint32_t* counts_host, int n);
/* The stride of the masked reset's bank rows for a bank of n_bank rows (-1 if n_bank < 1). */
int cbev_bank_stride(int n_bank);
/* Deferred canonical reset (off by default). With it on, cbev_reset_terminated
 * records the reset instead of launching it, and the next cbev_step of the same
 * records and frame ring folds it into its first kernel (k_ego; the envs take
 * the same bank rows, records and ring slots end up as cbev_reset_masked leaves
 * them, the mask is read when that step runs): the canonical loop's
 * step -> reset(reset_mask=terminated) -> step costs no reset launch. Any other
 * call on the context that reads or writes its state (every cbev_reset* call,
 * cbev_expand_obs, cbev_vector_obs, cbev_resize_obs, cbev_pack_frames,
 * cbev_bank_cursor, cbev_profile_raster, ...) or a cbev_step that cannot take
 * it first launches it on the stream it was recorded on, as does cbev_flush.
 * A caller that reads the records, the frame ring or writes the term buffer
 * itself calls cbev_flush first. Only records without actor slots (k_ego is the
 * step's first kernel) fold; otherwise cbev_reset_terminated launches at once.
 * The deferral is host-side state, taken when cbev_step is called: a cbev_step
 * captured into a graph while a reset is pending carries the folded reset, so
 * every replay resets the envs its term buffer selects at replay time (the mask
 * and the termination counts are read on the device); cbev_flush before capturing a
 * step that must not reset. Neither call allocates (safe under a global-mode
 * stream capture). */
int cbev_set_deferred_reset(cbev_ctx* ctx, int on);
/* 1 when a deferred reset is recorded and not yet applied. */
int cbev_reset_pending(const cbev_ctx* ctx);
/* Launch a recorded deferred reset (k_reset_mask) now; no-op otherwise. */
int cbev_flush(cbev_ctx* ctx);

/* Wrapper stack on the device (wrap_env, envs/__init__.py:62-83). `ring` holds
 * n_frames frames per env (uint8[n_frames][n][h][w], slot `head` the newest;
 * h x w = the cbev_set_obs_size size, the render size by default):
 *   kind 0: semantic one-hot (rgb_to_semantic.py:65-142) + FrameStack + Flatten
 *           -> float32[n][F*C][h][w]; channel_lut[id] = bitmask of channels set
 *   kind 3: semantic + FrameStack + VehicleTemporalFusionWrapper
 *           (rgb_to_semantic.py:152-166,275-301) -> float32[n][C+2][h][w]
 *   kind 4: semantic + FrameStack + WeightedVehicleHistoryWrapper
 *           (rgb_to_semantic.py:169-191,304-332) -> float32[n][C][h][w]
 *           (kinds 3/4: the vehicle channel is the bit channel_lut[CBEV_PX_VEHICLE]
 *           sets; n_frames >= 3)
 *   kind 1: grayscale (gymnasium GrayscaleObservation) + FrameStack
 *           -> uint8[n][F][h][w]; channel_lut[id] = gray value
 *   kind 5: FrameStack of a ring that already holds gray values (cbev_resize_obs
 *           with gray = 1) -> uint8[n][F][h][w]; channel_lut unused (may be NULL)
 *   kind 2: RGB (render(), no wrappers) -> uint8[n][S][S][3] of the newest
 *           render-size frame; channel_lut[id] = 0xRRGGBB
 * C = n_channels. */
int cbev_expand_obs(cbev_ctx* ctx, const uint8_t* ring, int n, int n_frames, int head, int kind, int n_channels,
                    const uint32_t* channel_lut_host, void* out, void* stream);

/* obs_mode "vector" (CarlaBEV.render, carlabev.py:237-244): out = float32[n][7],
 * [x, y, yaw, v] of the hero state + its Stanley set point [cx, cy, cyaw] at
 * target_idx (stanley_controller.py:140-148), from the records as they are now. */
int cbev_vector_obs(cbev_ctx* ctx, const void* records, int n, float* out, void* stream);

/* The multi-GPU frame gather's wire format (palette ids are
 * <= 15): packed = uint8[n][S*S/2], byte j of env e = frames[e][2j] |
 * frames[e][2j + 1] << 4. cbev_unpack_frames is the inverse. The reference has
 * no multi-process path (SyncVectorEnv, envs/__init__.py:116-119): this halves
 * the bytes the gather of the compact observation moves over xGMI. frames must be
 * 16-byte and packed 8-byte aligned (CBEV_EINVAL otherwise). */
int cbev_pack_frames(cbev_ctx* ctx, const uint8_t* frames, int n, uint8_t* packed, void* stream);
int cbev_unpack_frames(cbev_ctx* ctx, const uint8_t* packed, int n, uint8_t* frames, void* stream);

/* EnvConfig.fov_masked: FovRenderer's static corner mask (envs/fov.py:46-68,96-99)
 * applied by the raster (step and reset frames) after compose, before the ego
 * overlay. mask_host = uint8[S][S], 0xff where the output is blacked out, 0
 * elsewhere (carlabev_env_amd/fov_mask.py builds pygame's polygon fill); NULL
 * turns the mask off. Not stream-ordered: call it before queuing work. */
int cbev_set_fov_mask(cbev_ctx* ctx, const uint8_t* mask_host);

/* ResizeObservation(obs_size) (gymnasium; cv2.resize INTER_AREA) between the
 * render and the mask / grayscale wrappers (envs/__init__.py:62-67). Sets the
 * wrapped frame size h x w (<= size; h == w == size turns resizing off) and
 * builds the INTER_AREA tables. Not stream-ordered: call it before queuing work. */
int cbev_set_obs_size(cbev_ctx* ctx, int h, int w);

/* Resize n palette-id frames (uint8[n][S][S], e.g. cbev_step's output) to the
 * cbev_set_obs_size size, fused with the next wrapper's colour test:
 *   gray = 0: out byte = the palette id whose colour equals the resized RGB,
 *             else CBEV_PX_OFF_PALETTE (all semantic channels 0) -> expand kinds 0/3/4
 *   gray = 1: out byte = the grayscale value of the resized RGB -> expand kind 5
 * Envs with mask[e] == 0 are skipped (mask NULL = all). The frame is written to
 * n_out destinations out + k*out_stride (e.g. every slot of the ring on reset).
 * Returns CBEV_ESTATE when no resize is configured. */
int cbev_resize_obs(cbev_ctx* ctx, const uint8_t* frames, int n, const uint8_t* mask, int gray, uint8_t* out,
                    int n_out, int64_t out_stride, void* stream);

/* Kernel timing with HIP events recorded on the step's own stream around each
 * step kernel (used by bench.py for the roofline figure). cbev_profile(ctx, 1)
 * resets the counters and starts recording (up to 8192 steps);
 * cbev_profile_read synchronises on the last event and returns the summed
 * milliseconds of [k_actors, k_ego, k_raster] and the step count. */
int cbev_profile(cbev_ctx* ctx, int enable);
int cbev_profile_read(cbev_ctx* ctx, double* ms3, int64_t* steps);

/* Average duration of one k_raster launch over `reps` back-to-back launches on
 * `stream`, timed with two HIP events around the burst (bench.py's roofline
 * figure: the per-kernel events of cbev_profile also count each launch's
 * dispatch gap). It re-renders the observation of the current records, so
 * call it right after a cbev_step (which writes the render set-up and the
 * drawn target bits) and before any reset: `frames` then receives the bytes
 * that step wrote. Synchronises; writes the milliseconds per launch to *ms. */
int cbev_profile_raster(cbev_ctx* ctx, void* records, int n, uint8_t* frames, int reps, void* stream, double* ms);

#ifdef __cplusplus
}
#endif

#endif /* CBEV_H */
