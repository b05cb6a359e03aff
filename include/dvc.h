/*
 * dvc.h — C-ABI of the MI355X-native per-frame surveillance-compression worker.
 *
 * This is the drop-in boundary for the reference's per-frame hot loop. The
 * reference (carlozamu/dynamic-video-compression-surveillance, pure Python over
 * OpenCV 4.11) has no FFI of its own: its per-frame worker is the body of the
 * loop in
 *   frame_differencing.py:85-138   filter_and_dilate_movements(...)   (FD path)
 *   motion_compression_opt.py:65-101, 141-185                          (OF path)
 * and the Python host (dynamic-video-compression-surveillance_amd/) binds these
 * symbols with ctypes exactly where the reference calls cv2.* inside that loop.
 * Each entry point below names the reference lines it replaces.
 *
 * Conventions
 *  - Plain pointers and sizes only; no C++ or torch types cross this boundary.
 *  - Frames are packed 8-bit BGR, H rows of `pitch` bytes (pitch >= 3*W), i.e.
 *    what cv2.VideoCapture.read() yields (fd:87).
 *  - Every function returns DVC_OK (0) or a negative DVC_E_* status; the text of
 *    the last error on the calling thread is available from dvc_last_error().
 *    The Python host turns a negative status into logging.error(...) and an
 *    early return, mirroring the reference's try/except (fd:140-145).
 *  - A handle is single-threaded (one feed). Distinct handles may
 *    be driven from distinct host threads concurrently.
 *  - Unless DVC_FLAG_DEVICE_PTRS is set, frame/output pointers are host memory:
 *    pageable buffers are staged through two sets of pinned buffers owned by
 *    the handle (chunk c+1 goes up while chunk c computes and chunk c-1 comes
 *    down), page-locked ones (dvc_host_alloc) are DMA'd directly; with the flag
 *    they are device pointers on the handle's device (device-resident mode).
 *  - Frame rows: `pitch` bytes each (>= 3*W), every row readable in full. Any
 *    width and pitch are accepted; rows the kernels cannot read in place
 *    (pitch % 4, rows shorter than 3*roundup(W,4) bytes) are re-pitched on
 *    the device first.
 */
#ifndef DVC_H
#define DVC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define DVC_ABI_VERSION 7
#define DVC_MAX_BATCH 512

/* ---- status codes ---------------------------------------------------------- */
#define DVC_OK             0
#define DVC_E_INVALID     -1  /* bad argument / unsupported geometry           */
#define DVC_E_HIP         -2  /* a HIP runtime call failed                     */
#define DVC_E_STATE       -3  /* call out of order (e.g. step before prime)    */
#define DVC_E_NOMEM       -4  /* device or pinned allocation failed            */
#define DVC_E_UNSUPPORTED -5  /* parameter combination not implemented on GPU */
#define DVC_E_ODD_DCT     -6  /* a static block has an odd side > 1: cv2.dct
                                 raises "Odd-size DCT's are not implemented"
                                 (fd:122) and the reference loop stops
                                 (fd:140); see dvc_fd_step                     */

/* ---- flags ----------------------------------------------------------------- */
#define DVC_FLAG_DEVICE_PTRS 0x1u /* prime/step pointers are device pointers   */
#define DVC_FLAG_KTIMING     0x2u /* hipEvent-time every launch of the dominant
                                     (back) kernel; read with dvc_fd_ktime()    */
#define DVC_FLAG_KEEP_PLANES 0x4u /* keep the filtered / dilated masks of the
                                     last frame for dvc_fd_read_plane()        */
#define DVC_FLAG_JOIN_STREAM 0x8u /* join create's hip_stream even when it is
                                     NULL (= the legacy default stream);
                                     without the flag NULL means "no caller
                                     stream"                                    */
#define DVC_FLAG_OF_DIRECT_SUMS 0x10u /* OF: direct per-pixel 9x9 box sums instead
                                     of OpenCV's running sums (the default,
                                     FarnebackUpdateFlow_Blur's order)          */
#define DVC_FLAG_OUT_I420    0x20u /* FD: overlay and compressed frames are written
                                     as the encoder's 4:2:0 input instead of BGR:
                                     cvtColor(frame, COLOR_BGR2YUV_I420) of what
                                     fd:112 / fd:131 hand to VideoWriter.write —
                                     I420 frames of W*H*3/2 bytes (Y plane, then
                                     U and V planes of W/2 x H/2; out_stride >=
                                     W*H*3/2). block_size 4 or 8, W and H
                                     multiples of it (else DVC_E_UNSUPPORTED)  */

#define DVC_FLAG_FD_UNFUSED  0x40u /* FD: write the outputs in one k_out pass after
                                     the accumulated mask instead of the fused
                                     front's speculative static-block outputs +
                                     k_fix4 (same bytes; the fused form reads each
                                     frame from HBM once instead of twice. It
                                     applies to block_size 4, BGR frames or
                                     4:2:0 surfaces read in place, BGR outputs
                                     in 4-byte aligned rows; the
                                     environment variable DVC_FD_FUSED=0 sets
                                     this flag for every handle)                */

/* ---- frame formats (video I/O) ----------------------------- */
/* What the worker's frames are. The reference's are packed BGR straight from
 * cv2.VideoCapture.read() (fd:87); a hardware decoder (VCN via rocDecode) or a
 * Y4M file yields 4:2:0 YUV, which the worker converts on the GPU exactly as
 * cv2.cvtColor(COLOR_YUV2BGR_I420 / COLOR_YUV2BGR_NV12) does before the loop
 * body, so a decoded surface never round-trips through the host.
 * YUV frame layout: luma = `height` rows of `pitch` bytes; the chroma plane(s)
 * start chroma_rows * pitch bytes after the frame's first byte (chroma_rows >=
 * height, 0 = height: decoder surfaces pad the luma height); I420: U plane of
 * height/2 rows of pitch/2 bytes, V plane (chroma_rows/2) * (pitch/2) bytes after
 * U; NV12: one interleaved UV plane of height/2 rows of `pitch` bytes. A frame
 * spans pitch * chroma_rows * 3/2 bytes. Width and height even. */
#define DVC_FMT_BGR  0
#define DVC_FMT_I420 1
#define DVC_FMT_NV12 2

/* Standalone conversions (the decode / encode ends of the video I/O), n frames
 * frame_stride (YUV) / bgr_stride (BGR) bytes apart, on `device`:
 *   dvc_yuv420_to_bgr  cv2.cvtColor(COLOR_YUV2BGR_I420 or _NV12) — what
 *                      cv2.VideoCapture.read() hands the loop (fd:87, of:66,145)
 *   dvc_bgr_to_i420    cv2.cvtColor(COLOR_BGR2YUV_I420) — the 4:2:0 frame an
 *                      encoder takes from cv2.VideoWriter.write() (fd:112,131)
 * flags: DVC_FLAG_DEVICE_PTRS = device pointers, enqueued on hip_stream (NULL:
 * the default stream) and asynchronous; otherwise host pointers, synchronous. */
int dvc_yuv420_to_bgr(const uint8_t* yuv, size_t pitch, int fmt, int chroma_rows, int width, int height, int n,
                      size_t frame_stride, uint8_t* bgr, size_t bgr_pitch, size_t bgr_stride, int device,
                      void* hip_stream, uint32_t flags);
int dvc_bgr_to_i420(const uint8_t* bgr, size_t bgr_pitch, size_t bgr_stride, int width, int height, int n,
                    uint8_t* yuv, size_t pitch, int chroma_rows, size_t frame_stride, int device, void* hip_stream,
                    uint32_t flags);

/* ---- frame-differencing (FD) path ------------------------------------------ */

/*
 * Parameters, derived on the host from the reference kwargs of
 * filter_and_dilate_movements (fd:21-30):
 *   width,height  scaled frame size int(W*scale_factor), int(H*scale_factor) (fd:60-61),
 *                 any size >= 16 x 16.
 *   src_width,src_height  size of the frames handed to prime/step (the
 *                 video's, fd:57-58); 0 = width,height. When they differ the
 *                 worker resizes every frame on the GPU first (cv2.resize
 *                 INTER_LINEAR 8U, fd:74,91).
 *   block         block_size (fd:22), 1..128 (DVC_E_UNSUPPORTED above: a
 *                 static block's DCT planes are staged in LDS); partial blocks
 *                 at the right and bottom edges are their slices (fd:117-127).
 *   ithresh       floor(motion_threshold): cv::threshold on 8U floors the
 *                 threshold, so motion = absdiff > ithresh (fd:97).
 *   min_area2     floor(2*min_area): a contour is kept iff 2*area > min_area2,
 *                 which is contourArea(c) > min_area exactly, because 2*area of
 *                 an integer-vertex polygon is an integer (fd:103).
 *   ksize,anchor  dilation kernel np.ones((k,k)) with OpenCV's default anchor
 *                 k/2 (fd:80,106). 1 <= ksize <= 127 (DVC_E_UNSUPPORTED above:
 *                 a row is dilated by word shifts of at most 63 bits).
 *   alpha,beta,gamma  addWeighted weights as float32: release_factor,
 *                 1-release_factor, 0 (fd:107).
 *   quant         quantization_level as float32 (fd:123).
 *   prime_ksize,prime_sigma  GaussianBlur of frame 0: 25, 30.0 (fd:77).
 *   max_batch     frames per device launch (see the field).
 */
typedef struct dvc_fd_params {
    int32_t width;
    int32_t height;
    int32_t block;
    int32_t ithresh;
    int64_t min_area2;
    int32_t ksize;
    int32_t anchor;
    float alpha;
    float beta;
    float gamma;
    float quant;
    int32_t prime_ksize;
    double prime_sigma;
    uint32_t flags;
    uint32_t max_batch; /* 0/1..DVC_MAX_BATCH: frames one device launch covers in
                           dvc_fd_step_batch (longer calls are chunked). Bit
                           planes are allocated for three batches in flight, the
                           contour filter's working arrays for one (~20 MB per
                           1080p frame in all; ~8 GB at 383). */
    int32_t src_width;  /* 0: = width  */
    int32_t src_height; /* 0: = height */
    int32_t in_format;  /* DVC_FMT_BGR (0) / DVC_FMT_I420 / DVC_FMT_NV12: the frames
                           handed to prime/step (src size; YUV: `pitch` is the luma
                           pitch, frames converted on the GPU first, fd:87) */
    int32_t chroma_rows;/* YUV: see the frame layout above (0 = src_height) */
} dvc_fd_params;

/* Cumulative per-handle counters (all frames stepped since create/prime). */
typedef struct dvc_fd_stats {
    uint64_t frames;        /* frames stepped                                  */
    uint64_t motion_px;     /* pixels with absdiff > ithresh                   */
    uint64_t components;    /* external contours (fill-closed 8-components)    */
    uint64_t static_blocks; /* blocks whose accumulated mask is all zero       */
} dvc_fd_stats;

typedef struct dvc_fd dvc_fd;

/* Library / device introspection. */
int         dvc_abi_version(void);
const char* dvc_last_error(void);
int         dvc_device_count(int* count);

/* Page-locked host memory for frames and outputs: host-pointer steps DMA such
 * buffers directly (no staging copy on the CPU). The reference's frames come
 * from cv2.VideoCapture.read() (fd:87); a reader that decodes into these
 * buffers feeds the worker at PCIe rate. */
int  dvc_host_alloc(size_t bytes, void** out);
void dvc_host_free(void* p);

/* Create a feed handle on `device`. The stages run on four internal streams
 * (blur/threshold front, contour filter, dilate + accumulate, overlay/compress
 * output) with three batches' buffers in flight; only the two recurrences
 * (previous gray, accumulated mask) are serial. `hip_stream` (a hipStream_t or
 * NULL) is the caller's stream: when given, every prime/step call first waits
 * for the work queued on it before the call (e.g. the copy producing the
 * frames, reads of earlier outputs), and work queued on it after the call sees
 * the call's outputs — stream-ordered use without host syncs (calls on one
 * handle then do not overlap each other; with NULL they pipeline across calls
 * and dvc_fd_sync is the only ordering point). Device-pointer steps return
 * after enqueueing: dvc_fd_sync (or any read-back call) waits for all streams.
 * Replaces the per-video setup at fd:56-82. */
int dvc_fd_create(const dvc_fd_params* params, int device, void* hip_stream, dvc_fd** out);

/* Frame 0: resize (fd:74), gray (fd:75) + GaussianBlur(25x25, sigma 30) (fd:77)
 * -> previous gray; accumulated mask := 0 (fd:81). Resets the cumulative stats
 * and clears a DVC_E_ODD_DCT stop. Frames are src_width x src_height. */
int dvc_fd_prime(dvc_fd* h, const uint8_t* bgr, size_t pitch);

/* Resume a feed instead of priming it (checkpoint / resume): the state the
 * reference carries across frames — the previous blurred gray (fd:93,133)
 * and the accumulated mask (fd:107) — as host H*W planes (dvc_fd_read_plane's
 * DVC_PLANE_GRAY and DVC_PLANE_ACC export them). The next step continues
 * exactly as the uninterrupted run; counters restart as after dvc_fd_prime. */
int dvc_fd_set_state(dvc_fd* h, const uint8_t* prev_gray, const uint8_t* acc);

/* One frame of the hot loop, fd:91-133: gray, GaussianBlur 5x5, absdiff,
 * threshold, findContours/contourArea/drawContours filter, dilate, addWeighted,
 * red overlay (fd:110-111) and the mask-gated block DCT quantisation with the
 * YCrCb round trip (fd:115-130). Outputs (each nullable, packed BGR of pitch
 * 3*W unless noted):
 *   overlay     the frame written to dilated_motion_mask_video (fd:112)
 *   compressed  the frame written to compressed_final_video (fd:131)
 *   acc_out     the accumulated mask after this frame, H*W bytes (fd:107)
 * The call is asynchronous with respect to the host when DVC_FLAG_DEVICE_PTRS
 * is set (dvc_fd_sync before reading outputs or reusing the input); with host
 * pointers it returns after the outputs have landed.
 * DVC_E_ODD_DCT: the frame has a static block with an odd side > 1 (an odd
 * block_size, or an odd partial edge block): like the reference, whose
 * cv2.dct raises there (fd:122) and whose try/except ends the loop (fd:140),
 * the frame's overlay is valid (fd:112 comes first), its compressed frame is
 * not, it is not counted in the stats' `frames`, and the handle refuses
 * further steps until the next prime. With device pointers the stop is
 * detected on the device and reported by the next synchronising call
 * (dvc_fd_sync / dvc_fd_get_stats / the next host-pointer step). */
int dvc_fd_step(dvc_fd* h, const uint8_t* bgr, size_t pitch,
                uint8_t* overlay, uint8_t* compressed, uint8_t* acc_out);

/* n consecutive frames of the feed in one call (the reference loop fd:85-138
 * run n times): frame t at bgr + t*frame_stride (rows of `pitch` bytes), its
 * outputs at overlay/compressed + t*out_stride (rows of 3*W bytes; each
 * nullable). Results are identical to n dvc_fd_step calls. Device launches
 * cover max_batch frames each: the blur/threshold front and the dilate /
 * accumulate / compress back walk the frames in order per tile (prev_gray and
 * the accumulated mask stay on chip), the contour filter of every frame of the
 * batch runs as one grid, and batch i+1's front overlaps batch i's back.
 * Same synchronisation rules as dvc_fd_step; on DVC_E_ODD_DCT the stats'
 * `frames` counts the frames completed before the stopping one k (outputs
 * before k are complete, overlay k is valid). */
int dvc_fd_step_batch(dvc_fd* h, const uint8_t* bgr, size_t pitch, size_t frame_stride, int n,
                      uint8_t* overlay, uint8_t* compressed, size_t out_stride);

/* Wait for every launch of the handle. */
int dvc_fd_sync(dvc_fd* h);

/* Read the cumulative counters (synchronises the handle). */
int dvc_fd_get_stats(dvc_fd* h, dvc_fd_stats* out);

/* Debug/parity access to the internal planes of the LAST stepped frame, each
 * H*W bytes written to host memory: 0 gray (blurred, fd:93), 1 motion mask
 * {0,255} (fd:97), 2 filtered mask {0,255} (fd:101-104), 3 accumulated mask
 * (fd:107), 4 dilated mask {0,255} (fd:106). Plane 4 needs
 * DVC_FLAG_KEEP_PLANES. Synchronises the handle. */
#define DVC_PLANE_GRAY     0
#define DVC_PLANE_MOTION   1
#define DVC_PLANE_FILTERED 2
#define DVC_PLANE_ACC      3
#define DVC_PLANE_DILATED  4
int dvc_fd_read_plane(dvc_fd* h, int plane, uint8_t* host_dst);

/* With DVC_FLAG_KTIMING: total milliseconds and launch count of the dominant
 * HBM-bound kernel (one launch per batch: the fused front — gray, blur,
 * threshold and the speculative overlay / compressed frames — where the batch
 * ran it, else k_out: overlay + compress) since the last reset (synchronises
 * the handle). reset!=0 clears. */
int dvc_fd_ktime(dvc_fd* h, double* total_ms, uint64_t* launches, int reset);

/* Which kernel dvc_fd_ktime timed in the last batch: DVC_KTIME_OUT (k_out) or
 * DVC_KTIME_FRONT_FUSED (k_front with the fused outputs: block_size 4, BGR
 * frames in and out, 4-byte aligned output rows). Negative on error. */
#define DVC_KTIME_OUT 0
#define DVC_KTIME_FRONT_FUSED 1
int dvc_fd_ktime_kernel(const dvc_fd* h);

/* Batches of device frames (DVC_FLAG_DEVICE_PTRS, frames the kernels read in
 * place, no KTIMING; not a batch of > 128 frames whose outputs overlap a batch
 * still in flight, which takes the stage streams) run as one HIP graph launch
 * each: the
 * same kernels, arguments and dependencies as the stage streams, captured once
 * per slot and launch shape and re-parameterised per call (a call's host cost
 * drops from ~80 us to a graph launch). DVC_FD_GRAPH=0 in the environment at
 * create turns the path off. *batches: batches launched as graphs since
 * create, *builds: graphs built (both nullable). */
int dvc_fd_graph_stats(const dvc_fd* h, uint64_t* batches, uint64_t* builds);

void dvc_fd_destroy(dvc_fd* h);

/* The contour-area filter alone (fd:100-104) on an arbitrary host mask (H*W
 * bytes, nonzero = foreground): runs the same device kernels as dvc_fd_step
 * (run extraction, union-find, hole resolution, area, kept-mask paint) and
 * writes the filtered mask {0,255} to host memory. W, H >= 4.
 * *components (nullable) receives the number of external contours.
 * Synchronous; for the parity tests. */
int dvc_contour_filter(const uint8_t* mask, int width, int height, int64_t min_area2,
                       int device, uint8_t* filtered, uint64_t* components);

/* ---- optical-flow (OF) path ------------------------------------------------- */

/*
 * The per-frame worker of motion_compression_opt.py with its two passes fused
 * in memory: temporal_smoothing_flow (of:65-101) produces the rectangle mask of
 * frame t, compress_with_motion (of:141-185) compresses frame t with it. The
 * reference round-trips both through lossy mp4v files in between (of:99-100,
 * 121-122); the fused worker hands the exact mask and frame over instead.
 *   flow_threshold, alpha_fraction, window, morph_kernel  of:29-31 kwargs
 *                 (0.5, 0.2, 30, 2 as process_single_video_of passes, of:215-218)
 *   pyr_scale..poly_sigma  calcOpticalFlowFarneback arguments (of:72-81)
 *   quant         QTY_aggressive (100, of:138), 8x8 blocks on Y, Cr, Cb
 */
typedef struct dvc_of_params {
    int32_t width;
    int32_t height;
    float flow_threshold;
    float quant;
    double alpha_fraction;
    int32_t window;
    int32_t morph_kernel;
    double pyr_scale;
    int32_t levels;
    int32_t winsize;
    int32_t iterations;
    int32_t poly_n;
    double poly_sigma;
    uint32_t flags;      /* DVC_FLAG_DEVICE_PTRS | DVC_FLAG_KTIMING | DVC_FLAG_KEEP_PLANES */
    uint32_t max_batch;  /* 0/1..DVC_MAX_BATCH frames per device launch (see dvc_of_step_batch) */
    int32_t in_format;   /* DVC_FMT_BGR (0) / DVC_FMT_I420 / DVC_FMT_NV12 (of:66,145 read
                            BGR; 4:2:0 frames are converted on the GPU first) */
    int32_t chroma_rows; /* YUV: luma rows before the chroma plane(s), 0 = height */
} dvc_of_params;

typedef struct dvc_of dvc_of;

/* Cumulative per-handle counters (all frames stepped since prime). */
typedef struct dvc_of_stats {
    uint64_t frames;        /* frames stepped                                   */
    uint64_t motion_px;     /* pixels with |flow| > flow_threshold (of:82-83)   */
    uint64_t components;    /* 8-connected components of the smoothed mask
                               after close/open (one rectangle each, of:93-97)  */
    uint64_t static_blocks; /* full 8x8 blocks with an all-zero mask (of:161)   */
} dvc_of_stats;

/* Create an OF feed handle on `device` (GPU constraints, DVC_E_UNSUPPORTED
 * outside them: width and height >= 8, morph_kernel 1..64 (and its halo rows
 * within the LDS at that width), poly_n 5 or 7, winsize <= 17, window
 * 1..255, <= 6 pyramid levels). Replaces the per-video setup at
 * of:38-62. The gray/pyramid, flow and vote/morphology/output stages run on
 * three internal streams with two batches' rings in flight; `hip_stream`
 * (hipStream_t or NULL) is joined as in dvc_fd_create. Device-pointer steps
 * return after enqueueing: dvc_of_sync (or any read-back call) waits for all. */
int dvc_of_create(const dvc_of_params* params, int device, void* hip_stream, dvc_of** out);

/* Frame 0: gray (of:60) and its pyramid; the vote window is emptied (of:61). */
int dvc_of_prime(dvc_of* h, const uint8_t* bgr, size_t pitch);

/* Resume a feed instead of priming it (checkpoint / resume): the previous gray
 * (of:101) and the raw |flow| > thr masks of the last n frames, oldest first
 * (the deque of:84; only the newest `window` are kept), host H*W planes as
 * dvc_of_read_plane exports them (DVC_OF_PLANE_GRAY, DVC_OF_PLANE_RAW). The
 * next step continues exactly as the uninterrupted run; counters restart. */
int dvc_of_set_state(dvc_of* h, const uint8_t* prev_gray, const uint8_t* raw_masks, int n);

/* One frame of the fused worker: gray, calcOpticalFlowFarneback(prev, gray),
 * |flow| > thr, windowed vote, close/open, rectangle mask (of:70-97), and the
 * motion-gated compression of the same frame with that mask (of:151-183).
 *   mask        nullable, H*W bytes {0,255}: the frame written to mask.mp4 (of:99)
 *   compressed  nullable, packed BGR rows of 3*W: the frame written to
 *               compressed.mp4 (of:185)
 * Synchronisation as dvc_fd_step. */
int dvc_of_step(dvc_of* h, const uint8_t* bgr, size_t pitch, uint8_t* mask, uint8_t* compressed);

/* n consecutive frames (frame t at bgr + t*frame_stride): the pyramid, every
 * Farneback iteration, the morphology and the compression run as grids over
 * tiles x frames; only the vote walks the frames in order. Results identical
 * to n dvc_of_step calls. Mask t at mask + t*mask_stride, compressed frame t at
 * compressed + t*out_stride. */
int dvc_of_step_batch(dvc_of* h, const uint8_t* bgr, size_t pitch, size_t frame_stride, int n,
                      uint8_t* mask, size_t mask_stride, uint8_t* compressed, size_t out_stride);

int dvc_of_sync(dvc_of* h);
int dvc_of_get_stats(dvc_of* h, dvc_of_stats* out);

/* Planes of the LAST stepped frame, H*W bytes {0,255} (4: gray 0..255):
 * 0 |flow| > thr (of:83), 1 vote-smoothed (of:86), 2 after close/open
 * (of:89-90), 3 rectangle mask (of:93-97), 4 gray (of:71). */
#define DVC_OF_PLANE_RAW    0
#define DVC_OF_PLANE_SMOOTH 1
#define DVC_OF_PLANE_MORPH  2
#define DVC_OF_PLANE_RECT   3
#define DVC_OF_PLANE_GRAY   4
int dvc_of_read_plane(dvc_of* h, int plane, uint8_t* host_dst);

/* The Farneback flow of the last stepped frame, H*W*2 floats (dx, dy), to host
 * memory (of:72-81). Needs DVC_FLAG_KEEP_PLANES. */
int dvc_of_read_flow(dvc_of* h, float* host_dst);

/* With DVC_FLAG_KTIMING: total ms and launch count of the finest-level
 * Farneback iterations (k_flow at level 0, the dominant kernel). */
int dvc_of_ktime(dvc_of* h, double* total_ms, uint64_t* launches, int reset);

/* Which kernel ran the level-0 Farneback iterations of the last batch (what
 * dvc_of_ktime timed): DVC_KTIME_FLOW (k_flow: DVC_FLAG_OF_DIRECT_SUMS),
 * DVC_KTIME_FLOW_SCAN (the barrier-phased running-sum scan: winsize other than
 * 9) or DVC_KTIME_FLOW_SCAN2 (the pipelined scan, the reference's winsize 9).
 * Negative on error (DVC_E_STATE before the first step). */
#define DVC_KTIME_FLOW 2
#define DVC_KTIME_FLOW_SCAN 3
#define DVC_KTIME_FLOW_SCAN2 4
int dvc_of_ktime_kernel(const dvc_of* h);

void dvc_of_destroy(dvc_of* h);

/* Parity/debug readback of Farneback intermediates of the LAST stepped frame at
 * pyramid level `level` (host memory): what 0 = its polynomial expansion R
 * (h_k*w_k*5 floats), 1 = the previous frame's R, 2 = the flow after the first
 * iteration (h_k*w_k*2 floats; needs iterations >= 2 or level > 0). *w, *h
 * (nullable) receive the level size; dst may be NULL to query it. */
int dvc_of_debug_read(dvc_of* h, int what, int level, void* host_dst, int* w, int* hgt);

/* compress_with_motion for one frame with an arbitrary mask (of:141-185, e.g.
 * a decoded mask.mp4 frame): host pointers, synchronous. mask: H*W bytes,
 * nonzero = motion. Any W, H >= 1: partial 8x8 edge blocks are never
 * compressed (of:159,177) but take the YCrCb round trip (of:170-171). */
int dvc_of_compress(const uint8_t* bgr, size_t pitch, const uint8_t* mask, int width, int height, float quant,
                    int device, uint8_t* out);

/* compress_with_motion (motion_compression_opt.py:111-193) as a handle, n
 * frames per call: replaces the loop of:141-185 — its two reads (of:142-143),
 * the 3-channel mask's BGR2GRAY (of:147-149, exact: a coloured pixel can gray
 * to 0), the static full 8x8 blocks' DCT quantisation of Y, Cr, Cb, YCrCb->BGR
 * and per-block gray (of:151-183) — for frames t = 0..n-1:
 *   bgr + t*frame_stride      BGR rows of `pitch` (>= 3W)
 *   mask + t*mask_stride      mask rows of `mask_pitch`, mask_channels 1 (gray)
 *                             or 3 (BGR, as VideoCapture decodes mask.mp4)
 *   out + t*out_stride        compressed BGR rows of 3W (of:185)
 * Results identical to n dvc_of_compress calls (with the masks grayed).
 * quant = QTY_aggressive's constant (of:138, 100). Host pointers: synchronous
 * per call; DVC_FLAG_DEVICE_PTRS: device pointers, asynchronous on hip_stream
 * (NULL: the handle's own stream; dvc_ofc_sync waits). */
typedef struct dvc_ofc dvc_ofc;
int dvc_ofc_create(int width, int height, float quant, int max_batch, int device, void* hip_stream, uint32_t flags,
                   dvc_ofc** out);
int dvc_ofc_run(dvc_ofc* h, const uint8_t* bgr, size_t pitch, size_t frame_stride, const uint8_t* mask,
                size_t mask_pitch, size_t mask_stride, int mask_channels, int n, uint8_t* out, size_t out_stride);
int dvc_ofc_sync(dvc_ofc* h);
void dvc_ofc_destroy(dvc_ofc* h);

/* The Q8 fixed-point Gaussian taps OpenCV's bit-exact 8U GaussianBlur uses
 * (getGaussianKernelBitExact + error-diffusion rounding to 8 fraction bits).
 * n odd, 1 <= n <= 63. Exposed for the parity tests. */
int dvc_gaussian_taps_q8(int n, double sigma, uint16_t* taps);

/* ---- diagnostics ----------------------------------------------------------- */
/* Not a reference interface: the measurement bench.py quotes the FD roofline
 * against beside the 8 TB/s spec (SURVEY.md §8d "fraction of measured
 * stream-copy bandwidth on the same box"). A hand-written 16-B-per-lane copy
 * of `bytes` (use >> 256 MB, the Infinity Cache) repeated `reps` times on
 * `device`, nontemporal loads and stores if `nontemporal`; *gbps = bytes
 * read + written per second / 1e9. */
int dvc_copy_rate(int device, size_t bytes, int reps, int nontemporal, double* gbps);

#ifdef __cplusplus
}
#endif

#endif /* DVC_H */
