/*
 * kompressor_hip.h -- C-ABI of libkompressor_hip.so, the MI355X (gfx950) engine behind the
 * drop-in ``kompressor_amd.{image,volume}`` API.
 *
 * Conventions
 *   - Arrays are dense, C-contiguous, channels-last device buffers: volumes [B, D, H, W, C],
 *     images [B, H, W, C].  ``C`` is the product of all trailing (channel) dims.
 *   - Every entry point is stream-ordered on ``stream`` (a hipStream_t; NULL = legacy default
 *     stream), returns 0 on success or a negative kmp_status, and never synchronises the
 *     device, allocates, or frees memory (graph-capturable).  ``kmp_last_error()`` returns a
 *     thread-local message for the last failure.
 *   - Geometry follows the reference: an even spatial dim ``n`` is reflect-padded by one
 *     (``dims`` = 1), the lowres grid has L = (n + dims + 1) / 2 nodes, L - 1 cells, and the
 *     stored (trimmed) extent of node-lattice arrays is E = L - dims = ceil(n / 2).
 *
 * Each function names the reference interface it replaces (reference @ v1, file:line).  The
 * reference is pure Python on JAX: "replaces" means the Python function whose semantics the
 * kernel reproduces; the Python layer in kompressor_amd binds these through ctypes.
 */
#ifndef KOMPRESSOR_HIP_H
#define KOMPRESSOR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ihipStream_t* kmp_stream_t; /* ABI-identical to hipStream_t */

typedef enum {
  KMP_OK = 0,
  KMP_ERR_ARG = -1,      /* bad pointer, shape, dtype or enum */
  KMP_ERR_UNSUPPORTED = -2, /* valid request the engine does not implement */
  KMP_ERR_LAUNCH = -3,   /* HIP launch / runtime error */
} kmp_status;

typedef enum { KMP_U8 = 0, KMP_U16 = 1, KMP_I32 = 2, KMP_F32 = 3, KMP_U32 = 4 } kmp_dtype;

/* Residual coders, utils.py:28-55 (+ the build's mod-2^32 coder for bit-cast float32). */
typedef enum { KMP_CODER_RAW = 0, KMP_CODER_U8 = 1, KMP_CODER_U16 = 2, KMP_CODER_U32 = 3 } kmp_coder;
typedef enum { KMP_ENCODE = 0, KMP_DECODE = 1 } kmp_direction;

typedef enum {
  /* mean of the (2p+2)^d lowres neighbourhood, cast to the dtype, broadcast to all channels:
     the reference test predictor, tests/volume/test_encode_decode.py:43-55 */
  KMP_PRED_MEAN = 0,
  /* pred[k] = sum_n feat[n] * W[n, k] + b[k] in float32 (MFMA), cast to the dtype
     (build-defined; fills the reference's predictions_fn slot, volume/encode_decode.py:48) */
  KMP_PRED_LINEAR = 1,
  /* the same predictor on the matrix cores: bf16x2 split of features and weights, one
     v_mfma_f32_16x16x32_bf16 per chunk of 8 features (kmp_bf16x2.h); within the north star's 1e-5
     of the f64 value rather than bit-equal to the f32 fma chain; uint8 / uint16 samples */
  KMP_PRED_LINEAR_MFMA = 2,
} kmp_predictor_kind;

typedef struct {
  int32_t kind;         /* kmp_predictor_kind */
  int32_t padding;      /* neighbourhood padding p >= 0 */
  const float* weights; /* LINEAR: device [N, K] row-major, N = (2p+2)^d, K = 19 (3D) / 5 (2D) */
  const float* bias;    /* LINEAR: device [K] */
} kmp_predictor;

/* Sub-box of the output frame [0, E) per spatial axis (z, y, x; 2D uses y, x).  NULL = all.
   Used by the chunked drivers (encode_decode_chunk.py:77-117): a launch writes exactly the
   outputs whose block coordinate lies in the box. */
typedef struct {
  int64_t begin[3];
  int64_t end[3];
} kmp_region;

/* ---------------------------------------------------------------------------------------- */
/* Library                                                                                   */
/* ---------------------------------------------------------------------------------------- */
const char* kmp_version(void);
const char* kmp_last_error(void);
/* Name of the last kernel family this thread launched (e.g. "wave3d_encode", "fast3d_decode",
   "generic_encode"): lets tests and callers see which code path served a call. */
const char* kmp_last_launch(void);
/* 1 if the kernels were built for the device's ISA (gfx950) and a device is visible. */
int kmp_device_ok(void);

/* Process-wide dispatch options: switches to a fallback kernel family, the
   encode store policy, the block order.  Each starts from the environment variable of the same
   name, read once when the library loads; launches read the table, never the environment.
   ``kmp_set_option(name, value)`` sets one (KMP_ERR_ARG for an unknown name);
   ``kmp_clear_option`` returns it to the kernel's own default; ``kmp_get_option`` returns 1 and
   the value when set, 0 when unset, KMP_ERR_ARG for an unknown name.  Not part of the
   reference (which has no such switches); no production use needs them. */
int kmp_set_option(const char* name, int value);
int kmp_clear_option(const char* name);
int kmp_get_option(const char* name, int* value);

/* Device address of pinned (page-locked, device-mapped) host memory, for zero-copy streaming:
   the fused kernels then read the input from / write the outputs to host memory over the host
   link directly (kompressor_amd.stream, the reference's host-resident arrays,
   volume/encode_decode.py:30-85).  KMP_ERR_UNSUPPORTED if ``host`` is not such memory. */
int kmp_host_device_pointer(void* host, void** device);

/* ---------------------------------------------------------------------------------------- */
/* Fused encode / decode (one pass over HBM each).                                           */
/* ---------------------------------------------------------------------------------------- */

/* Replaces volume/encode_decode.py:30-56 ``encode`` for a built-in predictor and coder:
   pad_highres -> lowres_from_highres -> maps_from_highres -> predictor ->
   maps_from_predictions -> encode_fn per map -> trim.  ``highres`` [B, D, H, W, C] of
   ``dtype``; writes ``lowres_out`` [B, Ed, Eh, Ew, C] (dtype) and ``maps_out[7]`` in
   LR, UD, FB, C, Z, Y, X order with trimmed shapes (volume/utils.py:270-276) in the coder's
   dtype (RAW -> int32).  ``dims_out[3]`` receives the even-dim padding.  ``workspace`` must
   hold ``kmp_volume_workspace_bytes`` bytes (may be NULL when that is 0). */
int kmp_volume_encode(int32_t dtype, const void* highres, int64_t B, int64_t D, int64_t H, int64_t W,
                      int64_t C, const kmp_predictor* predictor, int32_t coder, void* lowres_out,
                      void* const maps_out[7], int32_t dims_out[3], const kmp_region* region,
                      void* workspace, size_t workspace_bytes, kmp_stream_t stream);

/* Replaces volume/encode_decode.py:59-85 ``decode``: pad_lowres/pad_maps -> predictor ->
   decode_fn per map -> highres_from_lowres_and_maps -> trim.  ``lowres`` [B, Ed, Eh, Ew, C],
   ``maps[7]`` as produced by kmp_volume_encode, ``dims[3]`` the even padding; writes
   ``highres_out`` [B, 2Ed-1+dd, 2Eh-1+dh, 2Ew-1+dw, C]. */
int kmp_volume_decode(int32_t dtype, const void* lowres, const void* const maps[7], int64_t B,
                      int64_t Ed, int64_t Eh, int64_t Ew, int64_t C, const int32_t dims[3],
                      const kmp_predictor* predictor, int32_t coder, void* highres_out,
                      const kmp_region* region, void* workspace, size_t workspace_bytes,
                      kmp_stream_t stream);

/* Bytes of device workspace the fused calls need for this shape/predictor (0 on the fast path). */
int64_t kmp_volume_workspace_bytes(int32_t dtype, int64_t B, int64_t D, int64_t H, int64_t W, int64_t C,
                                   const kmp_predictor* predictor);

/* 2D analogues: image/encode_decode.py:30-85; maps_out[3] in LR, UD, C order. */
int kmp_image_encode(int32_t dtype, const void* highres, int64_t B, int64_t H, int64_t W, int64_t C,
                     const kmp_predictor* predictor, int32_t coder, void* lowres_out,
                     void* const maps_out[3], int32_t dims_out[2], const kmp_region* region,
                     void* workspace, size_t workspace_bytes, kmp_stream_t stream);
int kmp_image_decode(int32_t dtype, const void* lowres, const void* const maps[3], int64_t B, int64_t Eh,
                     int64_t Ew, int64_t C, const int32_t dims[2], const kmp_predictor* predictor,
                     int32_t coder, void* highres_out, const kmp_region* region, void* workspace,
                     size_t workspace_bytes, kmp_stream_t stream);
int64_t kmp_image_workspace_bytes(int32_t dtype, int64_t B, int64_t H, int64_t W, int64_t C,
                                  const kmp_predictor* predictor);

/* ---------------------------------------------------------------------------------------- */
/* Primitives (the geometry API re-exported by volume/__init__.py:31-35, image/__init__.py)  */
/* ``nsp`` = number of spatial axes (2 = image, 3 = volume); ``shape`` holds them z,y,x      */
/* (image: y,x).                                                                            */
/* ---------------------------------------------------------------------------------------- */

/* volume/utils.py:77-80, image/utils.py:52-55: out = in[:, ::2, ::2(, ::2)] */
int kmp_lowres_from_highres(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3],
                            int64_t C, void* out, kmp_stream_t stream);

/* volume/utils.py:158-171, image/utils.py:89-96: the 7 (3) parity-class maps, untrimmed. */
int kmp_maps_from_highres(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3],
                          int64_t C, void* const out[7], kmp_stream_t stream);

/* volume/utils.py:37-74, image/utils.py:37-49: [B, cells..., 19 (5), C] training targets. */
int kmp_targets_from_highres(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3],
                             int64_t C, void* out, kmp_stream_t stream);

/* volume/utils.py:174-195, image/utils.py:99-116: interleave lowres [B, L..., C] and the
   7 (3) maps (shapes as maps_from_highres of a (2L-1)^d grid) into [B, 2L-1..., C]. */
int kmp_highres_from_lowres_and_maps(int32_t nsp, int32_t dtype, const void* lowres, const void* const maps[7],
                                     int64_t B, const int64_t lshape[3], int64_t C, void* out,
                                     kmp_stream_t stream);

/* volume/utils.py:199-210, image/utils.py:120-129: stack of the (2p+2)^d shifted windows of
   an already padded lowres [B, S..., C] -> [B, S-2p-1..., N, C]. */
int kmp_features_from_lowres(int32_t nsp, int32_t dtype, const void* lowres, int64_t B, const int64_t shape[3],
                             int64_t C, int32_t padding, void* out, kmp_stream_t stream);

/* volume/utils.py:83-155, image/utils.py:58-86: float32 aggregation of [B, cells..., K, C]
   predictions (K = 19 / 5) onto the 7 (3) maps, normalised, cast back to dtype. */
int kmp_maps_from_predictions(int32_t nsp, int32_t dtype, const void* preds, int64_t B, const int64_t cells[3],
                              int64_t C, void* const out[7], kmp_stream_t stream);

/* Mean predictor applied to a padded lowres window (the reference test predictor, as used by
   predictions_fn): == maps_from_predictions(repeat(mean(features_from_lowres(x, p)))) */
int kmp_mean_predict_maps(int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B,
                          const int64_t shape[3], int64_t C, int32_t padding, void* const out[7],
                          kmp_stream_t stream);

/* The same maps written as ``out_dtype``: the sample dtype, or KMP_F32 -- the values a
   float32-emitting predictions_fn (a network, volume/encode_decode.py:48) hands the coder; 3D,
   C == 1 windows only (else KMP_ERR_UNSUPPORTED). */
int kmp_mean_predict_maps_typed(int32_t nsp, int32_t dtype, int32_t out_dtype, const void* padded_lowres,
                                int64_t B, const int64_t shape[3], int64_t C, int32_t padding,
                                void* const out[7], kmp_stream_t stream);

/* Linear predictor on a padded lowres window: per-cell [B, cells..., K, C] predictions in the
   dtype (MFMA f32), optionally also the f32 pre-cast values (``preds_f32`` may be NULL). */
int kmp_linear_predict(int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B, const int64_t shape[3],
                       int64_t C, int32_t padding, const float* weights, const float* bias, void* preds_out,
                       float* preds_f32, kmp_stream_t stream);
/* the same for KMP_PRED_LINEAR_MFMA (kmp_bf16x2.h): the matrix-core arithmetic every fused kernel of
   that kind reproduces bit for bit; uint8 / uint16 samples */
int kmp_linear_predict_mfma(int32_t nsp, int32_t dtype, const void* padded_lowres, int64_t B, const int64_t shape[3],
                            int64_t C, int32_t padding, const float* weights, const float* bias, void* preds_out,
                            float* preds_f32, kmp_stream_t stream);

/* jnp.pad on the spatial axes (volume/utils.py:213-260, image/utils.py:132-178):
   mode 0 = 'symmetric', 1 = 'reflect'.  Negative pads crop (== trim, volume/utils.py:263-276). */
int kmp_pad(int32_t nsp, int32_t dtype, const void* in, int64_t B, const int64_t shape[3], int64_t C,
            const int64_t pad_lo[3], const int64_t pad_hi[3], int32_t mode, void* out, kmp_stream_t stream);

/* Box copy with dtype conversion -- the slicing and ``.at[box].set`` steps of the chunked
   driver (volume/encode_decode_chunk.py:101-115): for o in [0, ext) per spatial axis,
   out[b, out_off + o, c] = cast(in[b, in_off + o, c]).  Integer narrowing wraps; float -> int is
   the XLA truncating cast. */
int kmp_copy_box(int32_t nsp, int32_t in_dtype, const void* in, const int64_t in_shape[3], const int64_t in_off[3],
                 int32_t out_dtype, void* out, const int64_t out_shape[3], const int64_t out_off[3], int64_t B,
                 int64_t C, const int64_t ext[3], kmp_stream_t stream);

/* Tile split / reassembly for the batched metric workload (BASELINE configs C3/C4): the
   reference codes a batch of independent arrays along its leading axis (every primitive is
   [:, ...]-parallel, volume/utils.py:80,161-169); this turns ONE volume [D, H, W, C] (image
   [H, W, C]) into the batch [n, Tz, Ty, Tx, C] of its tiles in z-major tile order
   (direction 0) and back (direction 1).  Every extent must be a multiple of the tile's. */
int kmp_tiles(int32_t nsp, int32_t dtype, int32_t direction, const void* src, const int64_t shape[3], int64_t C,
              const int64_t tile[3], void* dst, kmp_stream_t stream);

/* Residual coders utils.py:28-55 on n elements.  ``pred_dtype``/``x_dtype`` are the operand
   dtypes (x = gt for ENCODE, encoded for DECODE); the output is uint8 / uint16 / int32 /
   uint32 for KMP_CODER_U8 / U16 / RAW / U32. */
int kmp_code(int32_t direction, int32_t coder, int32_t pred_dtype, const void* pred, int32_t x_dtype,
             const void* x, int64_t n, void* out, kmp_stream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* Callback path: an opaque predictions_fn with a built-in coder (kmp_callback.hip).  The    */
/* reference's steps on either side of the callback, fused; results identical to them.      */
/* ---------------------------------------------------------------------------------------- */

/* pad_neighborhood(lowres_from_highres(pad_highres(h)), p) (volume/encode_decode.py:36-48):
   the window encode hands predictions_fn, [B, L+2p..., C], straight from the highres. */
int kmp_window_from_highres(int32_t nsp, int32_t dtype, const void* highres, int64_t B, const int64_t shape[3],
                            int64_t C, int32_t padding, void* window_out, kmp_stream_t stream);

/* pad_neighborhood(pad_lowres(lowres, dims), p) (volume/encode_decode.py:70-76): the window
   decode hands predictions_fn, from the trimmed lowres [B, E..., C]. */
int kmp_window_from_lowres(int32_t nsp, int32_t dtype, const void* lowres, int64_t B, const int64_t shape[3],
                           int64_t C, const int32_t dims[3], int32_t padding, void* window_out, kmp_stream_t stream);

/* trim(lowres) and trim_maps([encode_fn(p, g) for p, g in zip(preds, maps_from_highres(
   pad_highres(h)))]) (volume/encode_decode.py:49-56) with encode_fn the built-in coder of the
   dtype: ``preds`` are predictions_fn's 7 (3) untrimmed maps in the sample dtype. */
int kmp_encode_with_predictions(int32_t nsp, int32_t dtype, int32_t coder, const void* highres, int64_t B,
                                const int64_t shape[3], int64_t C, const void* const preds[7], void* lowres_out,
                                void* const maps_out[7], kmp_stream_t stream);

/* trim(highres_from_lowres_and_maps(pad_lowres(lowres), [decode_fn(p, e) for p, e in
   zip(preds, pad_maps(maps))])) (volume/encode_decode.py:77-85), built-in decode_fn. */
int kmp_decode_with_predictions(int32_t nsp, int32_t dtype, int32_t coder, const void* lowres,
                                const void* const maps[7], int64_t B, const int64_t shape[3], int64_t C,
                                const int32_t dims[3], const void* const preds[7], void* highres_out,
                                kmp_stream_t stream);

/* The two above with the prediction maps' dtype given separately: ``pred_dtype`` is the sample
   dtype or KMP_F32 -- a network's float32 output, which the reference's coders read as
   jnp.int32(pred) (truncating; out-of-range saturates here), utils.py:28-55. */
int kmp_encode_with_predictions_typed(int32_t nsp, int32_t dtype, int32_t coder, int32_t pred_dtype,
                                      const void* highres, int64_t B, const int64_t shape[3], int64_t C,
                                      const void* const preds[7], void* lowres_out, void* const maps_out[7],
                                      kmp_stream_t stream);
int kmp_decode_with_predictions_typed(int32_t nsp, int32_t dtype, int32_t coder, int32_t pred_dtype,
                                      const void* lowres, const void* const maps[7], int64_t B, const int64_t shape[3],
                                      int64_t C, const int32_t dims[3], const void* const preds[7], void* highres_out,
                                      kmp_stream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* Bit-plane container payload (kmp_pack.hip; SURVEY.md §8f f-3 -- no reference counterpart, */
/* the reference returns the residual arrays unreduced, volume/encode_decode.py:56; format    */
/* spec: oracle/packing.py).  n samples of ``dtype`` (8/16/32-bit), zigzag-mapped, blocks of 64 */
/* stored as width 64-bit bit-planes.  ``workspace`` holds kmp_pack_workspace_bytes(n) bytes.  */
/* ---------------------------------------------------------------------------------------- */
int64_t kmp_pack_blocks(int64_t n);
int64_t kmp_pack_workspace_bytes(int64_t n);
/* byte offset in the workspace of the uint64 payload length (in 64-bit words) the plan writes */
int64_t kmp_pack_total_offset(int64_t n);
/* widths[nblocks] of x, and the block offsets + total payload words into the workspace */
int kmp_pack_plan(int32_t dtype, const void* x, int64_t n, uint8_t* widths, void* workspace, kmp_stream_t stream);
/* the payload (8-byte aligned) of x, after kmp_pack_plan on the same workspace */
int kmp_pack(int32_t dtype, const void* x, int64_t n, const uint8_t* widths, const void* workspace,
             uint64_t* payload, kmp_stream_t stream);
/* block offsets from stored widths, then the samples */
/* container header bytes written by a kernel (no host copy): dst[0:len) = bytes (len <= 128),  */
/* dst[zero_from:zero_to) = 0, and, when words_at >= 0, the u64 payload word count of the last    */
/* kmp_pack_plan on ``workspace`` (n samples) at dst + words_at -- stream-ordered after the plan */
int kmp_pack_header(uint8_t* dst, const uint8_t* bytes, int32_t len, int64_t zero_from, int64_t zero_to,
                    const void* workspace, int64_t n, int64_t words_at, kmp_stream_t stream);
int kmp_unpack_plan(const uint8_t* widths, int64_t n, void* workspace, kmp_stream_t stream);
int kmp_unpack(int32_t dtype, const uint64_t* payload, int64_t n, const uint8_t* widths, const void* workspace,
               void* out, kmp_stream_t stream);

/* ---------------------------------------------------------------------------------------- */
/* Block-adaptive Rice entropy coding of coded maps, bundle format v2 (kmp_rice.hip; SURVEY.md  */
/* §8f f-3 -- no reference counterpart, volume/encode_decode.py:56 returns the residuals         */
/* unreduced; byte layout spec: oracle/rice.py pack_bundle).  n samples of ``dtype`` (8/16/32-bit), */
/* zigzag-mapped, blocks of 64: params[b] = Rice k + 1 (0 = all-zero block), bw[b] = the block's  */
/* 32-bit payload words; tiles of 256 blocks.  All arrays of a bundle share ONE payload region in  */
/* tile order; each array keeps a u64 table of its tiles' word offsets into it.                  */
/* ---------------------------------------------------------------------------------------- */
typedef struct kmp_rice_array {
  const void* samples; /* encode: the input samples; decode: the output samples (written)      */
  int64_t n;           /* samples                                                                */
  int64_t side_off;    /* byte offset in the bundle of params[nb]; bw[nb] at side_off + pad8(nb)  */
  int64_t toff_off;    /* byte offset of the u64 tile offsets [kmp_rice_tiles(n)] (8-aligned)    */
  int64_t rec_off;     /* byte offset of the array's {u64 first word, u64 end word} (8-aligned)  */
} kmp_rice_array;
/* tiles of 256 blocks of 64 samples: ceil(ceil(n / 64) / 256) */
int64_t kmp_rice_tiles(int64_t n);
/* workspace of the single-pass encode: the look-back states of tiles_total tiles + a ticket */
int64_t kmp_rice_bundle_workspace_bytes(int64_t tiles_total);
/* one launch for ``count`` (<= 32) arrays of one dtype, whose tiles are global tiles           */
/* tile_begin .. + their count of the bundle's ``tiles_total``: samples read once, side          */
/* information / tile offsets / records / payload written into ``bundle`` (payload region at    */
/* byte payload_off); the tile of global index tiles_total - 1 writes the bundle's payload words */
/* (u64 at byte 56) and byte size (u64 at byte 64).  Calls for one bundle go in tile order on    */
/* one stream (replaces round 2's kmp_rice_plan / kmp_rice_pack and their two scan launches).   */
int kmp_rice_bundle_encode(int32_t dtype, const kmp_rice_array* arrays, int32_t count, int64_t tile_begin,
                           int64_t tiles_total, uint8_t* bundle, int64_t payload_off, void* workspace,
                           kmp_stream_t stream);
/* the inverse into each array's ``samples``: no scan launch (tile offsets from the table); side */
/* information checked in the same pass -- every read stays inside the tile's / payload's        */
/* extent, inconsistent tiles decode as zeros and add 1 to *bad (caller-zeroed device uint64)   */
/* (replaces round 2's kmp_unpack_plan + kmp_unpack_check + kmp_rice_unpack)                    */
int kmp_rice_bundle_decode(int32_t dtype, const kmp_rice_array* arrays, int32_t count, int64_t tile_begin,
                           const uint8_t* bundle, int64_t payload_off, uint64_t payload_words,
                           unsigned long long* bad, kmp_stream_t stream);

/* CRC-32 (zlib / IEEE: reflected 0xEDB88320, init and final xor 0xFFFFFFFF; == zlib.crc32) of   */
/* ``data`` into the device uint32 *crc_out (kmp_crc.hip): the container file's integrity check    */
/* (container.py; the reference has no file format, volume/encode_decode.py:56   */
/* returns arrays in memory).  ``n_max`` bytes are covered, or -- when ``n_dev`` is a device       */
/* int64 -- min(*n_dev, n_max), the length read by the kernel (a bundle's size field, no host sync). */
/* ``data`` 16-byte aligned.  One memset of *crc_out + one launch.                               */
int kmp_crc32(const uint8_t* data, int64_t n_max, const int64_t* n_dev, uint32_t* crc_out, kmp_stream_t stream);

/* Bit-plane side-information check (the planes format): count the blocks whose stored widths   */
/* no encoder produces (> W) -- format 0 -- or, format 1, Rice params / bw -- into the uint64 at  */
/* workspace + kmp_pack_total_offset(n) + 8, beside the payload length of the last scan          */
int kmp_unpack_check(int32_t format, int32_t dtype, const uint8_t* side_a, const uint8_t* side_b, int64_t n,
                     void* workspace, kmp_stream_t stream);

/* Categorical rank coder utils.py:58-111: ``logits`` float32 [n, L]; x/out of ``dtype`` [n]. */
int kmp_categorical(int32_t direction, const float* logits, int64_t n, int64_t L, int32_t dtype, const void* x,
                    void* out, kmp_stream_t stream);

#ifdef __cplusplus
}
#endif
#endif /* KOMPRESSOR_HIP_H */
