/*
 * zs_gpu.h -- C-ABI of the MI355X batched deflate/inflate engine
 * (libzsgpu.so, built from zlib-streams-ts_amd/csrc).
 *
 * The drop-in boundary for zlib-streams-ts's hot path.  Each batch entry runs
 * N independent streams, and stream i produces exactly the bytes (or the
 * error) that piping in[i] alone through the reference's web-streams layer
 * yields when the whole buffer is passed in ONE write() followed by close():
 *
 *   zs_deflate_batch*  replaces, per stream,
 *       new CompressionStream(format, {level})            src/mod/streams.ts:242-251
 *         -> createZeroCopyCompressionTransform           src/mod/streams.ts:216-228
 *         -> deflateInit2_(s, level, 8, wbits, 8, 0)      src/mod/deflate/deflate.ts:253-343
 *         -> deflate(s, Z_NO_FLUSH) per 32 KiB, deflate(s, Z_FINISH), deflateEnd
 *                                                         src/mod/deflate/deflate.ts:716-1013
 *   zs_inflate_batch*  replaces, per stream,
 *       new DecompressionStream(format)                   src/mod/streams.ts:253-262
 *         -> inflateInit2_(s, wbits) / inflate / inflateEnd
 *                                                         src/mod/inflate/inflate.ts:174-192,332-1185
 *   zs_crc32_batch / zs_adler32_batch replace           src/mod/common/crc32.ts:26-58,
 *                                                         src/mod/common/adler32.ts:4-25
 *
 * Conventions
 *   - Plain pointers and sizes only.  Buffers named d_* are device pointers
 *     (HBM) on the context's device; the per-stream layout arrays (offsets,
 *     lengths, capacities) are host arrays owned by the caller for the call.
 *   - wbits follows the format -> windowBits mapping of streams.ts:220,233:
 *     -15 "deflate-raw", 15 "deflate" (zlib), 31 "gzip", -16 "deflate64-raw"
 *     (inflate only).  level: 0..9 or -1 (= 6, deflate.ts:268-270).
 *   - Status codes are the reference's Z_* values (common/constants.ts:21-29).
 *     Per-stream status: ZS_STREAM_END on success; ZS_BUF_ERROR if out_cap[i]
 *     is too small (size outputs with zs_deflate_bound); decode errors as the
 *     reference reports them (see zs_inflate_batch_device).
 *   - Return value of every call: ZS_OK, or ZS_STREAM_ERROR for invalid
 *     arguments (the reference's deflateInit2_ validation, deflate.ts:281-294,
 *     which the stream layer reports as "init failed: -2", streams.ts:53), or
 *     ZS_MEM_ERROR when device memory cannot be obtained.  zs_last_error()
 *     describes the last failure on the calling thread.
 *   - Output offsets and capacities of the device entry points must be
 *     multiples of 4 bytes (the engine writes 32-bit words; ZS_STREAM_ERROR
 *     otherwise): no store leaves [out_off[i], out_off[i] + out_cap[i]).  The
 *     host-buffer entries take any inflate capacity (they round it up inside
 *     their own staging and copy back only the bytes produced).  Inputs may be
 *     packed at any byte offset.
 */
#ifndef ZS_GPU_H
#define ZS_GPU_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define ZS_OK 0
#define ZS_STREAM_END 1
#define ZS_NEED_DICT 2
#define ZS_STREAM_ERROR (-2)
#define ZS_DATA_ERROR (-3)
#define ZS_MEM_ERROR (-4)
#define ZS_BUF_ERROR (-5)

/* stream-layer phase of a per-stream failure (streams.ts:53,117,170) */
#define ZS_PHASE_NONE 0
#define ZS_PHASE_INIT 1
#define ZS_PHASE_PROCESS 2
#define ZS_PHASE_FINISH 3

typedef struct zs_ctx zs_ctx;

/* One context per device (one process per GPU).  Workspaces grow on demand
 * and are reused across calls; a context is not re-entrant across threads. */
int zs_ctx_create(int device, zs_ctx **out);
void zs_ctx_destroy(zs_ctx *ctx);
const char *zs_last_error(void);
const char *zs_version(void);

/* Re-checks the hardware property the fast chain builders use: same-address
 * LDS atomics of one wave instruction apply in lane order (gfx950).  Writes the
 * number of violations (0 expected).  zs_ctx_create runs it; when it does not
 * hold, the context uses the ballot-ranked builders instead (option lane_order
 * = 0, which can also be set by hand; the output bytes are the same).  No
 * reference counterpart (engine self-check). */
int zs_selftest(zs_ctx *ctx, uint64_t *violations);

/* deflateBound for a fresh stream with memLevel 8 (deflate.ts:615-674). */
uint64_t zs_deflate_bound(uint64_t source_len, int wbits);

/* Batched compression, device-resident buffers.  Enqueued on hip_stream (a
 * hipStream_t, or NULL for the context's own stream); returns once enqueued.
 * d_status[i] / d_out_len[i] (device int32 / uint32 arrays) are written. */
int zs_deflate_batch_device(zs_ctx *ctx, int level, int wbits, uint32_t n_streams, const uint8_t *d_in,
                            const uint64_t *in_off, const uint32_t *in_len, uint8_t *d_out, const uint64_t *out_off,
                            const uint32_t *out_cap, int32_t *d_status, uint32_t *d_out_len, void *hip_stream);

/* Same, host buffers: copies in, runs, copies out, synchronizes. */
int zs_deflate_batch(zs_ctx *ctx, int level, int wbits, uint32_t n_streams, const uint8_t *in, const uint64_t *in_off,
                     const uint32_t *in_len, uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                     int32_t *status, uint32_t *out_len);

/* Batched decompression, device-resident buffers.  Per stream: d_status[i]
 * (ZS_STREAM_END, or the Z_* code the stream layer reports), d_phase[i]
 * (ZS_PHASE_PROCESS / ZS_PHASE_FINISH for failures), d_msg[i] (index into
 * zs_inflate_message()), d_out_len[i], d_consumed[i] (input bytes used up to
 * the end of the stream; trailing bytes are ignored, streams.ts:74-76). */
int zs_inflate_batch_device(zs_ctx *ctx, int wbits, uint32_t n_streams, const uint8_t *d_in, const uint64_t *in_off,
                            const uint32_t *in_len, uint8_t *d_out, const uint64_t *out_off, const uint32_t *out_cap,
                            int32_t *d_status, int32_t *d_phase, int32_t *d_msg, uint32_t *d_out_len,
                            uint32_t *d_consumed, void *hip_stream);

int zs_inflate_batch(zs_ctx *ctx, int wbits, uint32_t n_streams, const uint8_t *in, const uint64_t *in_off,
                     const uint32_t *in_len, uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                     int32_t *status, int32_t *phase, int32_t *msg, uint32_t *out_len, uint32_t *consumed);

/* The same batch entries with the per-stream check value: check[i] is the
 * reference's strm.adler after stream i (deflate.ts:155-159,462,778,788;
 * inflate.ts:105,1014,1080): the adler32 (zlib) / crc32 (gzip) of the stream's
 * uncompressed bytes; for deflate-raw compression 1 (adler32(0), never updated
 * without a wrapper), for raw / deflate64-raw decompression 0 (createStream's
 * initial value, common/utils.ts:49); 0 for a stream that failed.  d_check /
 * check may be NULL (then these are the calls above). */
int zs_deflate_batch_device_ex(zs_ctx *ctx, int level, int wbits, uint32_t n_streams, const uint8_t *d_in,
                               const uint64_t *in_off, const uint32_t *in_len, uint8_t *d_out,
                               const uint64_t *out_off, const uint32_t *out_cap, int32_t *d_status,
                               uint32_t *d_out_len, uint32_t *d_check, void *hip_stream);
int zs_deflate_batch_ex(zs_ctx *ctx, int level, int wbits, uint32_t n_streams, const uint8_t *in,
                        const uint64_t *in_off, const uint32_t *in_len, uint8_t *out, const uint64_t *out_off,
                        const uint32_t *out_cap, int32_t *status, uint32_t *out_len, uint32_t *check);
int zs_inflate_batch_device_ex(zs_ctx *ctx, int wbits, uint32_t n_streams, const uint8_t *d_in,
                               const uint64_t *in_off, const uint32_t *in_len, uint8_t *d_out,
                               const uint64_t *out_off, const uint32_t *out_cap, int32_t *d_status, int32_t *d_phase,
                               int32_t *d_msg, uint32_t *d_out_len, uint32_t *d_consumed, uint32_t *d_check,
                               void *hip_stream);
int zs_inflate_batch_ex(zs_ctx *ctx, int wbits, uint32_t n_streams, const uint8_t *in, const uint64_t *in_off,
                        const uint32_t *in_len, uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                        int32_t *status, int32_t *phase, int32_t *msg, uint32_t *out_len, uint32_t *consumed,
                        uint32_t *check);

/* Unbounded decode, as DecompressionStream (streams.ts:46,132-182: pooled 64 KiB
 * output buffers until Z_STREAM_END, no output cap).  Host buffers; the outputs
 * land in ONE buffer the library allocates: on ZS_OK *out points to it, stream i
 * at (*out)[out_off[i]], out_len[i] bytes; release it with zs_free().  Members
 * are retried, alone, with eight times the room until they fit, so no member
 * reports the capacity message unless its output exceeds 4 GiB - 4 bytes (the
 * u32 length of this ABI). */
int zs_inflate_batch_auto(zs_ctx *ctx, int wbits, uint32_t n_streams, const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, uint8_t **out, uint64_t *out_off, int32_t *status, int32_t *phase,
                          int32_t *msg, uint32_t *out_len, uint32_t *consumed, uint32_t *check);
void zs_free(void *p);

/* Multi-GPU pool (SURVEY.md 8(b) "device mask", 8(e)): one context per device
 * of device_mask (bit d = HIP device d; 0 = every visible device).  A batch is
 * partitioned into contiguous stream ranges [k n / G, (k + 1) n / G) over the G
 * devices, one host thread per device; each shard writes straight into the
 * caller's arrays (offsets are absolute), so results are identical to one
 * device's.  Same arguments and semantics as the single-context host calls.
 * One batch at a time per pool. */
typedef struct zs_pool zs_pool;
int zs_pool_create(uint64_t device_mask, zs_pool **out);
/* The same from a list of devices, in shard order; a device may appear more
 * than once (each entry gets its own context: the pool's sharding rehearsed on
 * one GPU).  ZS_STREAM_ERROR for a device that does not exist. */
int zs_pool_create_list(const int *devices, int n_devices, zs_pool **out);
void zs_pool_destroy(zs_pool *pool);
int zs_pool_size(const zs_pool *pool);
int zs_pool_device(const zs_pool *pool, int k);
int zs_pool_deflate_batch(zs_pool *pool, int level, int wbits, uint32_t n_streams, const uint8_t *in,
                          const uint64_t *in_off, const uint32_t *in_len, uint8_t *out, const uint64_t *out_off,
                          const uint32_t *out_cap, int32_t *status, uint32_t *out_len, uint32_t *check);
int zs_pool_inflate_batch(zs_pool *pool, int wbits, uint32_t n_streams, const uint8_t *in, const uint64_t *in_off,
                          const uint32_t *in_len, uint8_t *out, const uint64_t *out_off, const uint32_t *out_cap,
                          int32_t *status, int32_t *phase, int32_t *msg, uint32_t *out_len, uint32_t *consumed,
                          uint32_t *check);
int zs_pool_inflate_batch_auto(zs_pool *pool, int wbits, uint32_t n_streams, const uint8_t *in,
                               const uint64_t *in_off, const uint32_t *in_len, uint8_t **out, uint64_t *out_off,
                               int32_t *status, int32_t *phase, int32_t *msg, uint32_t *out_len, uint32_t *consumed,
                               uint32_t *check);

/* The z_stream message for a d_msg index (inflate.ts:397-1031, inffast.ts:108,197,210). */
const char *zs_inflate_message(int32_t msg_index);

/* Per-stream checksums, check[i] = crc32(seeds[i], in[i]) / adler32(seeds[i], in[i])
 * with the reference's semantics (common/crc32.ts:26-58, common/adler32.ts:4-25):
 * the seed is a running checksum being continued; an empty stream returns the
 * seed unchanged.  seeds: host array of n_streams values, or NULL for the
 * initial values (crc32 0, adler32 1).  The _device forms take device buffers
 * and write d_check on the device (asynchronously on hip_stream); the host forms
 * take host buffers and return when check[] is filled. */
int zs_crc32_batch_device(zs_ctx *ctx, uint32_t n_streams, const uint8_t *d_in, const uint64_t *in_off,
                          const uint32_t *in_len, const uint32_t *seeds, uint32_t *d_check, void *hip_stream);
int zs_adler32_batch_device(zs_ctx *ctx, uint32_t n_streams, const uint8_t *d_in, const uint64_t *in_off,
                            const uint32_t *in_len, const uint32_t *seeds, uint32_t *d_check, void *hip_stream);
int zs_crc32_batch(zs_ctx *ctx, uint32_t n_streams, const uint8_t *in, const uint64_t *in_off,
                   const uint32_t *in_len, const uint32_t *seeds, uint32_t *check);
int zs_adler32_batch(zs_ctx *ctx, uint32_t n_streams, const uint8_t *in, const uint64_t *in_off,
                     const uint32_t *in_len, const uint32_t *seeds, uint32_t *check);

/* Kernel timing of the batch calls made on this context since the last query
 * (HIP events on the streams the kernels ran on; the calls themselves never
 * wait for them, the query does): device milliseconds from the first call's
 * start to the last call's end, and the summed duration of the named phase
 * ("sweep", "parse", "trees", "emit", "fast", "inflate_lane", ...).  Returns -1
 * when no timing is available. */
double zs_last_batch_ms(zs_ctx *ctx);
/* Members of the last inflate batch that the lane-per-member path decoded
 * (the rest went through the exact stream-layer state machine).  Synchronizes
 * the batch's stream.  For tests and tuning. */
uint32_t zs_last_inflate_lane_count(zs_ctx *ctx);
/* Members of the last inflate batch that the segmented decode finished
 * (inflate_seg.hip; the others of its members went on to the wave kernel).
 * Synchronizes.  For tests and tuning. */
uint32_t zs_last_inflate_seg_count(zs_ctx *ctx);
double zs_last_phase_ms(zs_ctx *ctx, const char *phase);
void zs_set_timing(zs_ctx *ctx, int on);
/* Engine options: "timing" (0/1, as zs_set_timing); "inflate_fast" (default 1):
 * decode members lane-per-member and re-run only those that do not end cleanly
 * on the exact stream-layer state machine (0: exact path for every member);
 * "check_phases" (default 0): synchronise after every kernel phase and fail
 * with ZS_MEM_ERROR naming the phase whose launch or execution failed;
 * "match_sweep" (default 1): levels 4..9 find matches by a counting sort by
 * hash + lock-step sweep, longer streams in windows of 65,535 positions with a
 * 32 KiB look-back (0: the chain-link + per-tile walk kernels, for every stream
 * -- a cross-check);
 * "lane_block" (default 0 = by batch size;
 * else 1..64, a power of two): members per workgroup of the inflate lane path;
 * "inflate_wave_min" (default 32768; 0 = never): members with more input bytes
 * are "large" and decode beside the lane kernel (side stream): deflate64 (and
 * raw deflate with inflate_ref_wrap 0) by the split decode (inflate_split.hip:
 * cut at block boundaries, pieces in parallel), the other formats one per wave
 * (inflate_wave.hip) or, when a batch has lane_large_min of them or more, one
 * per lane (the lane kernel's large-member instance) -- both track the
 * reference's inflate() calls and so reproduce the window-wrap copy below;
 * "inflate_split" (default 1; 0: large deflate64 members take the wave kernel);
 * "lane_large_min" (default 2304; 0: never): large-member count from which the
 * lanes replace the wave kernel;
 * "parse_waves" (default 0 = two below 2048 streams, else one; 1, 2 or 4):
 * waves per stream of the levels 4..9 lazy parse (two: 512-position segments,
 * two rounds' speculative passes at once);
 * "fast_group" (default 1): levels 1..3 replay deflate_fast a group of 64
 * positions at a time from speculative per-lane chain walks (0: step by step);
 * "lane_order" (default 1 when the self-test passes, else 0 and 1 is refused):
 * the chain builders rank equal hashes by same-address LDS atomics applying in
 * lane order (1) or by ballots (0);
 * "inflate_seg" (default 1): batches of at most "seg_small_batch" (default
 * 16,384) members decode every member with more than "seg_small_min" (default
 * 4096) input bytes -- and, in any batch, every member over inflate_wave_min --
 * by the segmented decode (inflate_seg.hip: blocks walked in order, each cut
 * across 64 lanes, the reference's calls tracked per piece); large deflate64
 * members and high-expansion members (cap > 64 KiB, >= 8 output bytes per
 * input byte) take the split / wave decoders instead; "seg_bits" (1024..8192,
 * default 0 = 4096 for members of >= 64 KiB of input on average, else 2048):
 * input bits per lane of an entry's first block; "seg_wide"
 * (default 1): the 2048-bit sync window for a batch of few large members;
 * "seg_split" (0 off, 1 on, default 2 = batches of at most 2 large members per CU):
 * each piece is cut in two at the first symbol start past its lane's middle, so
 * the decode runs twice the pieces, each half as long;
 * "seg_big_bits" (>= 65536, default 2^21): members with more input bits also
 * walk from the block starts a finder kernel proposes (more walks per member);
 * "seg_scratch_mb" (default 16384): the segmented decode's u16 scratch per
 * batch (2 bytes per byte of capacity); members past it take the other paths.
 * These options never change output bytes.  "inflate_ref_wrap" (default 1)
 * does: 1 reproduces the reference's inflate_fast window-wrap copy
 * (inffast.ts:133-147), which changes the output of members whose match
 * crosses the reference's window wrap between inflate() calls; 0 decodes with
 * zlib semantics (the bytes the compressor was given). */
int zs_set_option(zs_ctx *ctx, const char *name, int value);

/* Introspection for tests: copy an intermediate array of stream s of the last
 * deflate batch to host memory (what: 0 chain links u16/position, 1 match table
 * u32x2/position, 2 symbols u32, 3 block records, 4 stream record).  Returns
 * the bytes copied (0 if unavailable).  Synchronizes the device. */
uint64_t zs_debug_fetch(zs_ctx *ctx, int what, uint32_t s, void *dst, uint64_t cap);

/* Synthetic workload: kind 0 = T-corpus text,
 * 1 = M-corpus mixed, 2 = xorshift bytes; stream i uses seed
 * 0x9e3779b9 ^ (first_index + i).  Fills host memory with n_streams x len. */
void zs_corpus(int kind, uint32_t first_index, uint32_t n_streams, uint32_t len, uint8_t *out, int threads);

#ifdef __cplusplus
}
#endif
#endif
