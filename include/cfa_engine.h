/*
 * cfa_engine.h — C-ABI of libcfa.so, the MI355X (gfx950) consensus-reduction engine.
 *
 * This is the drop-in boundary for the CFA / CFA-GE neighbour-model mixing step of
 * labRadioVision/federated. The reference computes that step with numpy AXPY chains
 * inside its `consensus` package. Each entry point below replaces one of those chains
 * (citations are `path:line` under the reference tree; TF1 = tensorflow1_implementations,
 * TF2 = tensorflow2_implementations/MNIST_dataset unless stated).
 *
 * Conventions
 *   - Plain pointers and sizes only. Buffers are caller-owned device pointers
 *     (hipMalloc / PyTorch-ROCm tensors). The library allocates no device memory on the hot
 *     path (scratch comes from the caller, e.g. the gradient workspace; the one exception is
 *     cfa_mix_tf1_f32 above CFA_MAX_FANIN neighbours, documented there, whose caller-scratch
 *     form is cfa_mix_tf1_ex_f32). The host-only MQTT
 *     payload codec allocates its parse tree in host memory (freed by cfa_payload_free).
 *   - `stream` is a hipStream_t passed as void*; NULL means the legacy default stream.
 *     Every compute call is asynchronous on that stream. Every device pointer of a call must be
 *     memory of the stream's GPU: the library does not query pointer attributes on the launch
 *     path, so another GPU's pointer is not refused here (the Python engine refuses such
 *     tensors, federated_amd/engine.py _same_device).
 *   - Return 0 on success, a negative CFA_E* code on failure. `cfa_last_error()` returns a
 *     thread-local message for the last failure on the calling thread. No exceptions cross
 *     the ABI. Calls are re-entrant and thread-safe. The one piece of process-wide state is the
 *     host copy pool behind the host mix entry below, whose workers are created on first use and
 *     never destroyed: one call owns it at a time, and a concurrent call copies on its own thread.
 *   - `P` is the bucket length in fp32 elements. A "bucket" is one model (or gradient)
 *     flattened layer by layer, in the order the reference passes its tensors.
 *   - Pointer arrays (`nbrs`, `alphas`, `coeff`, `s`, `g`) are HOST arrays whose entries are
 *     device pointers (or host scalars for coefficients).
 *   - `out` may alias `local` / `W` (in-place update). Outputs must not alias any neighbour.
 *   - Any fan-in n >= 0 is accepted; n > CFA_MAX_FANIN is executed as several passes.
 *   - hipGraph capture: call cfa_device_prepare(device) once per device before capturing. After
 *     it, no entry point issues a device-attribute query, a kernel-attribute change or an
 *     allocation on the launch path (cfa_mix_tf1_f32 above CFA_MAX_FANIN refuses capture and
 *     points to cfa_mix_tf1_ex_f32), so captures run in the strict (global) mode.
 *
 * Where the ABI departs from the signatures sketched in SURVEY.md §8(b), entry by entry
 * (tests/test_capi.py holds the sketch's parameter lists and checks every prototype below
 * against this list)
 *   - cfa_mix_f32(out, local, nbrs, coeff, n, P, stream): `coeff` and `n` are SWAPPED relative to
 *     the sketch's (out, local, nbrs, n, coeff, P, stream), so that every mix entry reads
 *     (out, local, nbrs, <per-neighbour host array>, n, P, ...) alike: cfa_mix_seq_f32 and
 *     cfa_mix_seq_div_f32 take alphas (and divisors) in that same slot. A C caller following the
 *     sketch must swap the two. The sequential rule is its own entry (alphas, not closed-form
 *     coefficients) because the reference's fp32 chain is three roundings per step, which no
 *     coefficient vector reproduces.
 *   - cfa_mewma_update_f32(W, s, g, g_stride, n, rho, lr1, lr2, lr_split, init, use_filtered, P,
 *     stream) against the sketch's (W, s, g, n, rho, lr, use_filtered, P, stream):
 *     `g_stride` (per-neighbour element stride of g_j, NULL = contiguous) reads the
 *     `[..., devices]` gradient slices the sketch gave to cfa_mix_strided_f32; `rho` is a double
 *     so rho and 1 - rho each round once to fp32 as numpy does with a Python float; the one `lr`
 *     becomes (lr1, lr2, lr_split) because the reference applies -l1 to the layer-1 tensors and
 *     -l2 to the layer-2 tensors of one bucket (federated_sample_CNN_CFA-GE.py:16-17,29-30);
 *     `init` selects the 4-stage epoch-1 rule s_j <- g_j (cfa_ge_2stage.py:332-336).
 *   - cfa_compress_epilogue_f32(y, ref, mode, P, kept_count, stream) against the sketch's
 *     (y, ref_or_null, thr, rep, mode, kept_count, P, stream): `mode` replaces (thr, rep), since
 *     the four (thr, rep) pairs are fixed by cfa_ongraphs.py:225-273 and the mode also selects the
 *     sparse vs DPCM test, which (thr, rep) alone cannot express (a mode makes an inconsistent
 *     triple unrepresentable); `P` comes before `kept_count`, the order of every sized entry here.
 *   - cfa_mix_population_f32(out_ptrs, src_ptrs, csr_ptr, csr_idx, csr_coef, D, rule, P, stream)
 *     against (out_stack, in_stack, csr_ptr, csr_idx, csr_coeff, D, P, stream): device tables of
 *     bucket pointers instead of dense stacks, because a population's devices live in separate
 *     buffers (ping-pong models, halo rows, per-device allocations from callers) and a pointer
 *     table serves all of them with one launch (a dense [D, P] stack is the special case,
 *     cfa_mix_ring_round_f32); `rule` added so one launch serves the sequential CFA rule and the
 *     linear FedAvg form.
 *   - cfa_comm_init(comm, rank, nranks, id, device) against (rank, nranks, id, comm): the
 *     communicator out parameter comes first and `device` is added, so a caller thread need not
 *     have selected the GPU beforehand; the return value stays the status code.
 *   - cfa_mix_strided_f32 is not provided. The `[..., devices]` gradient slices of CFA-GE
 *     (cfa_ge_2stage.py:594-606) arrive in host memory (loadmat), and the host mixer gathers slot
 *     `ii` while packing the pinned staging rows, so every GPU read is a coalesced row. Read on
 *     the device, a stride-D slice pulls a whole line per 4 useful bytes: the round-1 entry ran at
 *     0.31 of peak with 2.5x over-fetch, so it was retired in round 2 (g_stride above keeps the
 *     strided read for the MEWMA update, whose caller may hold such slices on the device).
 *   - cfa_halo_exchange_f32, whose parameters the sketch elides, takes whole buckets; it is joined by
 *     cfa_p2p_group_f32, with per-message counts, for the routed, chunked halo.
 *     cfa_allreduce_scaled_f32 became cfa_allreduce_sum_f32 / cfa_reduce_sum_f32 because the
 *     pre-scaling is fused into the mix that produces the buffer (one pass fewer).
 *   - cfa_comm_destroy, cfa_last_error and cfa_version are as sketched.
 */
#ifndef CFA_ENGINE_H
#define CFA_ENGINE_H

#include <stddef.h>
#include <stdint.h>

#if defined(__GNUC__)
#define CFA_API __attribute__((visibility("default")))
#else
#define CFA_API
#endif

#ifdef __cplusplus
extern "C" {
#endif

#define CFA_VERSION 10000 /* 1.0.0 */
#define CFA_MAX_FANIN 16  /* neighbours folded per kernel pass */

enum {
  CFA_OK = 0,
  CFA_E_INVALID = -1,     /* bad argument (null pointer, negative size, bad mode) */
  CFA_E_HIP = -2,         /* HIP runtime error (launch, memcpy, device) */
  CFA_E_RCCL = -3,        /* RCCL error */
  CFA_E_UNSUPPORTED = -4, /* feature not available in this build */
  CFA_E_TIMEOUT = -5      /* a host-side wait gave up (cfa_host_wait_word) */
};

/* Mixing rules. */
enum {
  /* Sequential CFA rule: w <- w + a_j * (x_j - w), j = 0..n-1, evaluated as
   * t = x_j - w; t = a_j * t; w = w + t (three fp32 roundings, no FMA contraction).
   * This reproduces the fp32 numpy chain bit for bit. */
  CFA_RULE_SEQUENTIAL = 0,
  /* Linear combination: out = c_0 * local + sum_j c_{j+1} * x_j (fp32 FMA chain). */
  CFA_RULE_LINEAR = 1,
  /* Sequential rule with a divisor: w <- w + (a_j * (x_j - w)) / d_j (FedAvg form). */
  CFA_RULE_SEQUENTIAL_DIV = 2,
  /* Accumulation: w <- w + a_j * x_j, one rounding per product and per sum (fp64 fold only). */
  CFA_RULE_ACCUMULATE = 3
};

/* Compression epilogue modes (TF1/consensus/cfa_ongraphs.py:225-273). The fp32 entry points
 * (cfa_mix_seq_compress_f32, cfa_compress_epilogue_f32) evaluate them as numpy 2 does on fp32
 * arrays: threshold and replacement cast to fp32, test / product / DPCM sum in fp32. The TF1
 * entry points (cfa_mix_tf1_f32, cfa_mix_tf1_f64) evaluate them in fp64 on the fp64 chain, as
 * the reference does on its promoted W_up_l2. */
enum {
  CFA_COMPRESS_NONE = 0,
  CFA_COMPRESS_SPARSE = 1,          /* |y| < 1e-3 -> sign(y) * 1e-4                       :227-237 */
  CFA_COMPRESS_SPARSE_DPCM = 2,     /* |y - ref| < 1e-4 -> ref + sign(y - ref) * 1e-4      :239-249 */
  CFA_COMPRESS_SPARSE_DPCM_HI = 3,  /* |y - ref| < 1e-3 -> ref + sign(y - ref) * 1e-3      :250-260 */
  CFA_COMPRESS_SPARSE_HI = 4        /* |y| < 1e-2 -> sign(y) * 1e-3                        :261-271 */
};

CFA_API int cfa_version(void);
CFA_API const char* cfa_last_error(void);

/* Caches `device`'s CU count and LDS size and raises the gradient kernels' dynamic-LDS limit on
 * it, so that later launches query nothing (required before a strict hipGraph capture). The
 * calling thread's current device is restored. Idempotent. */
CFA_API int cfa_device_prepare(int device);

/* ---------------------------------------------------------------------------------------
 * (f2) MATLAB level-5 files of the TF1 exchange (host only). Every TF1 consensus call publishes
 * its model with scipy.io.savemat and loads its neighbours' with scipy.io.loadmat
 * (TF1/consensus/cfa.py:108-117, 131-139; cfa_ongraphs.py:214-223, 282-291;
 * cfa_ge_2stage.py:537-606). cfa_mat_write writes the bytes scipy's level-5 writer writes for real
 * numeric matrices (uncompressed, column-major data, 8-byte padding, small-data elements at <= 4
 * bytes); cfa_mat_read parses such files (scipy's or MATLAB's, uncompressed, little-endian,
 * real numeric classes only) and returns CFA_E_UNSUPPORTED for anything else, so the caller can
 * fall back to scipy. The parsed file owns the memory its variables point into.
 */
#define CFA_MAT_MAX_DIM 8
typedef struct {
  const char* name;
  int mat_class;   /* mxDOUBLE_CLASS = 6, SINGLE 7, INT8 8, UINT8 9, INT16 10, UINT16 11, INT32 12,
                      UINT32 13, INT64 14, UINT64 15 */
  int mi_type;     /* stored element type: miINT8 1, miUINT8 2, miINT16 3, miUINT16 4, miINT32 5,
                      miUINT32 6, miSINGLE 7, miDOUBLE 9, miINT64 12, miUINT64 13 */
  int ndim;
  int64_t dims[CFA_MAT_MAX_DIM];
  const void* data; /* column-major elements of mi_type */
  size_t nbytes;
} cfa_mat_var_t;
typedef struct cfa_mat cfa_mat_t;
CFA_API int cfa_mat_read(const char* path, cfa_mat_t** out);
CFA_API void cfa_mat_free(cfa_mat_t* mat);
CFA_API int cfa_mat_num_vars(const cfa_mat_t* mat);
CFA_API const cfa_mat_var_t* cfa_mat_vars(const cfa_mat_t* mat);
CFA_API const char* cfa_mat_header(const cfa_mat_t* mat);
CFA_API int cfa_mat_write(const char* path, const char* header, int nvars, const cfa_mat_var_t* vars);

/* ---------------------------------------------------------------------------------------
 * (f2) numpy files of the TF2 exchange (host only). The TF2 consensus / parameter-server modules
 * load each neighbour's status archive and model with np.load(..., allow_pickle=True)
 * (TF2/MNIST_dataset/consensus/consensus_v3.py:82-141, consensus_v4.py:30-95,
 * parameter_server_v2.py:83-164): results/dump_train_variables{k}.npz (np.savez, stored zip of
 * numeric .npy members) and results/dump_train_model{k}.npy (np.save of a 1-D object array of
 * per-layer ndarrays, i.e. a pickle). cfa_npy_read reads one file and locates its arrays in place:
 * a numeric .npy (kind CFA_NPY_ARRAY, one array), an object .npy whose pickle holds only numpy's
 * ndarray reconstructors and numeric elements (CFA_NPY_OBJECT, one array per element; nothing in
 * the file is executed), or a stored .npz of numeric members (CFA_NPY_ARCHIVE, CRC-checked, one
 * array per member, named without ".npy"). Anything else returns CFA_E_UNSUPPORTED (fall back to
 * np.load); truncated or corrupt files return CFA_E_INVALID. The parsed file owns the memory its
 * arrays point into.
 */
#define CFA_NPY_MAX_DIM 32
enum { CFA_NPY_ARRAY = 0, CFA_NPY_OBJECT = 1, CFA_NPY_ARCHIVE = 2 };
typedef struct {
  const char* name;   /* archive member name (without ".npy"); NULL for .npy files */
  const char* descr;  /* numpy dtype string: "<f4", "<f8", "<i8", "|b1", "|u1", ... */
  int itemsize;
  int ndim;
  int64_t shape[CFA_NPY_MAX_DIM];
  int fortran_order;
  const void* data;   /* elements in C order, or Fortran order when fortran_order */
  size_t nbytes;
} cfa_npy_array_t;
typedef struct cfa_npy cfa_npy_t;
CFA_API int cfa_npy_read(const char* path, cfa_npy_t** out);
/* The same on a file image already in memory; the arrays point into `image`, which the caller
 * keeps alive until cfa_npy_free. */
CFA_API int cfa_npy_parse(const void* image, size_t nbytes, cfa_npy_t** out);
CFA_API void cfa_npy_free(cfa_npy_t* npy);
CFA_API int cfa_npy_kind(const cfa_npy_t* npy);
CFA_API int cfa_npy_num_arrays(const cfa_npy_t* npy);
CFA_API const cfa_npy_array_t* cfa_npy_arrays(const cfa_npy_t* npy);

/* (f2) The drop-in host path of one mix as a native chunk pipeline: the local model and n
 * neighbour models arrive as per-layer fp32 arrays in pageable host memory (TF2
 * consensus_v3.py:144-157 over the loaded .npy layer lists; parameter_server_v2.py:159-161) and
 * the result goes back into per-layer arrays. The bucket range is cut into chunks of
 * chunk_elems; chunk c of every model is copied into `staging` (pinned host, chunk-major, slices
 * padded to 4 elements) by `threads` host threads while the kernel of chunk c - 1 reads its
 * slices over PCIe in place; each chunk's result lands in `out_pinned` (pinned host, P elements)
 * and is copied into out_layers as soon as its kernel is done. Each chunk runs cfa_mix_seq_f32
 * when divisors is NULL, else cfa_mix_seq_div_f32, so the result equals the single-shot mix
 * bit for bit. in_layers is model-major: model m (0 = local), layer k at
 * [m * L + k]. Returns when every output layer is written.
 * On an error return no kernel of the call is still running (the stream is drained), and the
 * host copy threads have left the caller's arrays, so they may be released; the one exception is
 * a host copy that has not finished 10 minutes after the pool's 30 s limit (the message says
 * "still copying"): the arrays passed to that call must then be kept alive.
 * cfa_host_mix_staging_elems gives the staging size one call needs. */
CFA_API size_t cfa_host_mix_staging_elems(const size_t* layer_elems, int L, int n, size_t chunk_elems);
CFA_API int cfa_host_mix_f32(float* const* out_layers, const float* const* in_layers,
                             const size_t* layer_elems, int L, int n, const float* alphas,
                             const float* divisors, float* staging, size_t staging_elems,
                             float* out_pinned, size_t chunk_elems, int threads, void* stream);

/* Host-path helpers (the per-call drop-in path): hipStreamSynchronize, and a
 * stream-ordered fetch of a device uint64 counter (e.g. a compression kept_count) into host
 * memory (pinned, for an asynchronous copy) followed by resetting the counter to zero; and one
 * asynchronous copy (the pinned staging of a batch of inputs). */
CFA_API int cfa_stream_synchronize(void* stream);
/* hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, stream): the staging copy of the host path. */
CFA_API int cfa_memcpy_async(void* dst, const void* src, size_t bytes, void* stream);
CFA_API int cfa_counter_fetch(unsigned long long* counter, unsigned long long* host_dst, void* stream);
/* Completion of a short call without hipStreamSynchronize's wake-up: cfa_stream_signal enqueues
 * a one-lane kernel that stores `value` into the 32-bit word `word_dev` (the device address of a
 * pinned host word, cfa_host_device_pointer) with a system-scope release, after the stream's
 * earlier work; cfa_wait_signal spins on the host word (acquire loads) until it reads `value`.
 * After spin_us microseconds without it, cfa_wait_signal falls back to hipStreamSynchronize(stream),
 * which also reports any error of the stream's work, and then requires the value. At the C1 call
 * shape this completes 3.5 us sooner than hipStreamSynchronize (profiles/r03v_flag_sync.jsonl).
 * The caller gives each concurrent user its own word and changes `value` at every call. */
CFA_API int cfa_stream_signal(unsigned* word_dev, unsigned value, void* stream);
CFA_API int cfa_wait_signal(const unsigned* word_host, unsigned value, void* stream, long long spin_us);

/* Host lane of the routed halo (federated_amd/hostlane.py): part of a round's halo travels
 * D2H over the sender's PCIe link into shared pinned host memory and H2D over the receiver's,
 * beside the xGMI links. cfa_host_register / cfa_host_unregister pin (hipHostRegister, mapped and
 * portable) and release a caller-mapped host range, e.g. a shared-memory segment both ranks map.
 * The sender raises a chunk's sequence number with cfa_stream_signal after its D2H copy (stream
 * ordered); the receiver's HOST thread waits for it with cfa_host_wait_word and only then enqueues
 * the H2D copy, so no wait ever parks on a GPU queue (a parked wait would hold every stream sharing
 * its hardware queue). cfa_host_wait_word polls the host word (acquire loads) until it reaches
 * `value` in sequence order ((int)(word - value) >= 0): it spins ~20 us, then sleeps in 20 us
 * steps, and returns CFA_E_TIMEOUT after `timeout_us` (> 0) without it. Host only: no HIP call. */
CFA_API int cfa_host_register(void* host, size_t bytes);
CFA_API int cfa_host_unregister(void* host);
CFA_API int cfa_host_wait_word(const unsigned* word_host, unsigned value, long long timeout_us);

/* The receive side of a host lane as a pump: one native host thread per lane walks a round's
 * operations in order. Each operation: wait until the host word `wait_word` reaches `wait_value`
 * (NULL: no wait; the same poll as cfa_host_wait_word, `timeout_us` per wait); copy `bytes` from
 * `src` to `dst` (0: none); raise `signal_word` to `signal_value` (NULL: none); record `event` (a
 * hipEvent_t, NULL: none) on the lane's stream; publish `mark` (> 0) as the round's progress.
 * GPU mode (`host_mode` 0): copies are hipMemcpyAsync on `stream`, signals cfa_stream_signal on it
 * (`signal_word` a device address), so nothing waits on a GPU queue and the caller's thread does not
 * wait either until it needs a group's rows. Host mode (1): memcpy and a release store into the host
 * word (no HIP call; the CPU tests). cfa_lane_pump_submit copies the list and returns at once
 * (CFA_E_INVALID while the previous round is still in progress); cfa_lane_pump_wait blocks until
 * `mark` has been published (mark < 0: the whole round) and returns CFA_E_TIMEOUT after
 * `timeout_us` without it. A wait of the pump that times out ends the round: that error is then
 * returned by every later wait and submit (sticky). cfa_lane_pump_destroy stops the thread
 * (interrupting a wait) and frees the pump. One caller thread per pump. */
typedef struct cfa_lane_op {
  const unsigned* wait_word;
  unsigned wait_value;
  unsigned signal_value;
  unsigned* signal_word;
  void* dst;
  const void* src;
  size_t bytes;
  void* event;
  int mark;
} cfa_lane_op;
CFA_API int cfa_lane_pump_create(void** pump, void* stream, int device, int host_mode);
CFA_API int cfa_lane_pump_submit(void* pump, const cfa_lane_op* ops, int n_ops, long long timeout_us);
CFA_API int cfa_lane_pump_wait(void* pump, int mark, long long timeout_us);
CFA_API int cfa_lane_pump_destroy(void* pump);

/* ---------------------------------------------------------------------------------------
 * (a1/a2/a5/a6) Sequential CFA mix of one device with n neighbours.
 *   out[i] = fold_j( w <- w + alphas[j] * (nbrs[j][i] - w) ), w0 = local[i]
 * Replaces:
 *   TF1/consensus/cfa.py:66-76 (per-neighbour loop :119-130, alpha = eps/N)
 *   TF1/consensus/cfa_ongraphs.py:109-119 (loop :196-213, alpha = eps/(1+n))
 *   TF1/consensus/cfa_mobilenet.py:82-91, cfa_ge_2stage.py:73-83 (stage 1, :449-466)
 *   TF2 consensus_v3.py:153-155 / consensus_v2.py:153-155 / consensus_v4.py:211-213 (weights)
 *   TF2 consensus_v3.py:236-238 / consensus_v4.py:251-253 (gradients)
 *   TF2/FL_over_MQTT/learner_consensus.py:150-153 (alpha = 1/2)
 * Bytes moved: (n + 2) * P * 4.
 */
CFA_API int cfa_mix_seq_f32(float* out, const float* local, const float* const* nbrs,
                    const float* alphas, int n, size_t P, void* stream);

/* Launch configuration of the streaming mix kernels (performance only; results are identical
 * for every configuration). */
typedef struct {
  int blocks_per_cu;  /* grid = min(tiles, CUs * blocks_per_cu); 0 = one workgroup per tile */
  int vec_per_lane;   /* 16-byte vectors per lane per bucket per tile: 1, 2, 4; 0 = auto */
  int nontemporal;    /* 1 = nontemporal (streaming) loads/stores for once-touched buckets */
} cfa_launch_t;

/* cfa_mix_seq_f32 with an explicit launch configuration (NULL = library default, from sweeps on
 * placement-calibrated buckets: one workgroup per CU and 2 vectors per lane, 1 for 3-5
 * neighbours; from 512K to 1.5M elements four workgroups per CU with 1 vector per lane, from 1.5M
 * to 8M four with 4 (up to 9 neighbours; with 2 below 3M above that); an explicit configuration
 * with vec_per_lane = 0 takes round 1's auto width). */
CFA_API int cfa_mix_seq_ex_f32(float* out, const float* local, const float* const* nbrs,
                               const float* alphas, int n, size_t P, const cfa_launch_t* launch,
                               void* stream);

/* (f1) FedAvg / parameter-server fold: w <- w + (alphas[j] * (nbrs[j] - w)) / divisors[j],
 * j = 0..n-1, each step rounded like numpy's `p + u*(x - p)/C` (fp32 multiply, then IEEE fp32
 * division by the count). Replaces TF2 parameter_server_v2.py:159-161 / parameter_server.py:154,
 * :74 (metalearning), FL_over_MQTT/PS_server.py:127-134, learner_consensus.py:150-153. */
CFA_API int cfa_mix_seq_div_f32(float* out, const float* local, const float* const* nbrs,
                                const float* alphas, const float* divisors, int n, size_t P,
                                void* stream);

/* Linear-combination mix: out[i] = coeff[0]*local[i] + sum_j coeff[j+1]*nbrs[j][i].
 * The closed form of the sequential rule (c_0 = prod(1-a_j), c_{j+1} = a_j prod_{k>j}(1-a_k)),
 * and the FedAvg / parameter-server aggregation shape
 * (TF2 parameter_server_v2.py:159-161, PS_server.py:127-134). */
CFA_API int cfa_mix_f32(float* out, const float* local, const float* const* nbrs,
                const float* coeff, int n, size_t P, void* stream);

/* Sequential mix fused with the compression epilogue of cfa_ongraphs.py:225-273.
 * The epilogue applies to elements [cbegin, cend) of the bucket (the W2 tensor), with
 * `local` as the DPCM reference (n_W_l2 is the pre-mix local, :246-247). The number of
 * elements in that range NOT replaced is ADDED to *kept_count (a device uint64; zero it
 * first). Mode CFA_COMPRESS_NONE adds (cend - cbegin). */
CFA_API int cfa_mix_seq_compress_f32(float* out, const float* local, const float* const* nbrs,
                             const float* alphas, int n, size_t P, int mode, size_t cbegin,
                             size_t cend, unsigned long long* kept_count, void* stream);

/* (a3) Standalone compression epilogue, in place on y[0..P), reference `ref` (may be NULL
 * for modes 1/4). Adds the kept count to *kept_count (device uint64). */
CFA_API int cfa_compress_epilogue_f32(float* y, const float* ref, int mode, size_t P,
                              unsigned long long* kept_count, void* stream);

/* (a1/a2/a3) TF1 mix with the reference's numpy-2 numerics, fp32 buckets in and out:
 *   step 0:  w = (double)local + alphas[0] * (double)(x_0 - local)   (x_0 - local in fp32)
 *   step j:  w = w + alphas[j] * ((double)x_j - w)                     (fp64)
 *   out = (float)w after the optional compression epilogue, evaluated on the fp64 w with the
 *   fp32 `local` as DPCM reference, on elements [cbegin, cend).
 * In the reference, eps * wf is an np.float64, so the first subtraction is fp32 and the rest of
 * the chain is promoted to fp64 (TF1/consensus/cfa.py:69-76, cfa_ongraphs.py:112-119 and the
 * compression loop :225-273, cfa_mobilenet.py:82-91, cfa_ge_2stage.py:76-83). The result is
 * the reference's fp64 result rounded once to fp32, which is what the TF1 drivers feed back
 * into their fp32 graph. alphas[j] = eps * wf_j are host doubles. kept_count (device uint64)
 * may be NULL only when mode == CFA_COMPRESS_NONE (no epilogue, no count); otherwise the
 * number of elements of [cbegin, cend) NOT replaced is ADDED to it, as in
 * cfa_mix_seq_compress_f32 (mode 0: cend - cbegin). n > CFA_MAX_FANIN chains passes through an fp64 scratch bucket
 * (8 * P bytes, stream-ordered allocation), so the result still rounds once. That allocation
 * cannot be captured: under hipGraph capture with n > CFA_MAX_FANIN this entry fails
 * (CFA_E_INVALID) and cfa_mix_tf1_ex_f32 must be used. */
CFA_API int cfa_mix_tf1_f32(float* out, const float* local, const float* const* nbrs,
                            const double* alphas, int n, size_t P, int mode, size_t cbegin,
                            size_t cend, unsigned long long* kept_count, void* stream);

/* The same TF1 chain over fp32 buckets, written UNROUNDED into an fp64 `out` (P doubles): the
 * fp64 arrays the reference itself returns when its inputs are fp32 (cfa.py:66-76 under numpy 2:
 * fp32 first subtraction, fp64 after; the epilogue in fp64). Equal to cfa_mix_tf1_f64 on the
 * widened buckets with step0_f32 = 1, at half the input bytes. n >= 1; passes above
 * CFA_MAX_FANIN chain in `out` itself (no scratch, no allocation). `out` (8 * P bytes) must not
 * overlap `local` or any neighbour (CFA_E_INVALID). */
CFA_API int cfa_mix_tf1_wide_f32(double* out, const float* local, const float* const* nbrs,
                                 const double* alphas, int n, size_t P, int mode, size_t cbegin,
                                 size_t cend, unsigned long long* kept_count, void* stream);

/* cfa_mix_tf1_f32 with a caller-owned fp64 scratch bucket (device, >= P doubles, 8-byte
 * aligned; used only when n > CFA_MAX_FANIN, may be NULL otherwise): no allocation at all. */
CFA_API int cfa_mix_tf1_ex_f32(float* out, const float* local, const float* const* nbrs,
                               const double* alphas, int n, size_t P, int mode, size_t cbegin,
                               size_t cend, unsigned long long* kept_count, double* scratch,
                               void* stream);

/* (a1-a4) TF1 mix on fp64 buckets: the reference's own TF1 arithmetic, with no rounding to fp32.
 * Under numpy 2 the reference's chain is fp64 (eps * wf is an np.float64) over whatever arrays
 * the caller and the .mat files hold, and it returns fp64 arrays. The buckets here are those
 * arrays widened to fp64 (exact for fp32 values):
 *   step 0:  w = local + alphas[0] * d,  d = step0_f32 ? (double)((float)x_0 - (float)local)
 *                                                     : x_0 - local
 *   step j:  w = w + alphas[j] * (x_j - w)
 * step0_f32 = 1 when the reference's local and first-neighbour arrays are both fp32 (numpy
 * subtracts them in fp32). The optional compression epilogue (cfa_ongraphs.py:225-273) is
 * applied in fp64 on [cbegin, cend) with `local` as DPCM reference; kept_count as in
 * cfa_mix_tf1_f32. Replaces TF1/consensus/cfa.py:69-76, cfa_ongraphs.py:112-119 + 225-273,
 * cfa_mobilenet.py:82-91, cfa_ge_2stage.py:76-83 (stage 1 of CFA-GE). */
CFA_API int cfa_mix_tf1_f64(double* out, const double* local, const double* const* nbrs,
                            const double* alphas, int n, int step0_f32, size_t P, int mode,
                            size_t cbegin, size_t cend, unsigned long long* kept_count,
                            void* stream);

/* (f1) fp64 fold of the reference's server-side chains, on fp64 buckets (fp32 arrays widened
 * exactly), one fp64 rounding per operation, w0 = local:
 *   CFA_RULE_SEQUENTIAL      w <- w + alphas[j] * (x_j - w)
 *   CFA_RULE_SEQUENTIAL_DIV  w <- w + (alphas[j] * (x_j - w)) / divisors[j]
 *   CFA_RULE_ACCUMULATE      w <- w + alphas[j] * x_j
 * Replaces the aggregation loops embedded in the reference's drivers, whose operands are fp64:
 *   TF2/FL_over_MQTT/PS_server.py:130-133 (SEQUENTIAL_DIV over the decoded fp64 payloads),
 *   TF2/FL_over_MQTT/learner_consensus.py:151-152 (SEQUENTIAL_DIV, u = 1, C = 2),
 *   TF1/federated_sample_CNN_CFA_FA.py:86-89 (ACCUMULATE from zeros, a = 1/devices),
 *   :103-110 and :130-133 (SEQUENTIAL, a = eps/devices), :280-283 (client, SEQUENTIAL, a = eps2).
 * `divisors` is read only by SEQUENTIAL_DIV. out may alias local. */
CFA_API int cfa_fold_f64(double* out, const double* local, const double* const* nbrs,
                         const double* alphas, const double* divisors, int n, int rule, size_t P,
                         void* stream);

/* (a4) CFA-GE MEWMA on fp64 buckets with the reference's numpy-2 operations
 * (cfa_ge_2stage.py:331-371, :593-621), for j = 0..n-1 in order:
 *   s_j <- init ? g_j : rho*g_j + (1-rho)*s_j
 *   W   <- W - lr(i) * (use_filtered ? s_j : g_j),  lr(i) = i < lr_split ? lr1 : lr2
 * The buckets hold the reference's arrays widened to fp64; f32_mask says which of them are fp32
 * arrays there (CFA_TF1_*_F32). rho, 1-rho and lr are Python floats in the reference, so each
 * product is computed in its array's dtype, a sum/difference is fp32 only when both operands
 * are, and a state is rounded to its array's dtype on store (as numpy's slice assignment does).
 * W and s_j are updated in place; g_j is read with element stride g_stride (NULL = all 1). */
enum { CFA_TF1_STATE_F32 = 1, CFA_TF1_GRAD_F32 = 2, CFA_TF1_W_F32 = 4 };
CFA_API int cfa_mewma_tf1_f64(double* W, double* const* s, const double* const* g,
                              const int64_t* g_stride, int n, double rho, double lr1, double lr2,
                              size_t lr_split, int init, int use_filtered, int f32_mask, size_t P,
                              void* stream);

/* (a4) CFA-GE gradient-bucket update (MEWMA), for j = 0..n-1 in order:
 *   s_j <- init ? g_j : rho*g_j + (1-rho)*s_j
 *   W   <- W - lr(i) * (use_filtered ? s_j : g_j),   lr(i) = i < lr_split ? lr1 : lr2
 * Replaces TF1/consensus/cfa_ge_2stage.py:593-621 (fast; CNN use_filtered=1, 2NN 0) and
 * :329-371 (4-stage: init=1 at epoch 1, use_filtered=0). W and s_j are updated in place.
 * g_j is read with element stride g_stride (1 = contiguous). rho is a double so that rho and
 * (1 - rho) are each rounded once to fp32, as numpy does with a Python-float hyperparameter.
 * Bytes moved: (3n + 2) * P * 4. */
CFA_API int cfa_mewma_update_f32(float* W, float* const* s, const float* const* g,
                         const int64_t* g_stride, int n, double rho, float lr1, float lr2,
                         size_t lr_split, int init, int use_filtered, size_t P, void* stream);

/* (e/f4) Sliding-window population pass: nb (1..8) consecutive devices of a ring window with hl
 * neighbours below and hr above (0..4 each), mixed with the sequential rule in one launch that
 * loads each row of the window once: (nb + hl + hr) * P * 4 bytes read and nb * P * 4 written,
 * against nb * (hl + hr + 2) * P * 4 for nb separate mixes, with identical results.
 *   rows[0 .. nb+hl+hr-1]: HOST table of device pointers, consecutive devices g0-hl .. g0+nb-1+hr
 *                          (the caller resolves ring wrap-around and halo rows);
 *   device b (0 <= b < nb) mixes local rows[b+hl] with rows[b .. b+hl-1] then
 *                          rows[b+hl+1 .. b+hl+hr] (the window order of cfa.py:14-32 /
 *                          consensus_v4.py:133-137), coefficient alphas[b] at every step (the
 *                          reference's eps policies give a window device one value:
 *                          1/(K+1), consensus_v3.py:145; eps*b/(b + m*b), cfa.py:66-68);
 *   out[0 .. nb-1]: HOST table of output device pointers (must not alias any row). */
CFA_API int cfa_mix_window_f32(float* const* out, const float* const* rows, const float* alphas,
                               int nb, int hl, int hr, size_t P, void* stream);

/* (e/f4) A whole ring-window round of a STACKED population in one launch: device d's model is
 * in + d * pitch (P floats), its output out + d * pitch; every device mixes with the ring window
 * [d-hl .. d-1, d+1 .. d+hr] (mod D) in that order with coefficient alphas[d] (DEVICE array of D
 * floats) at each step. The devices run as cfa_mix_window_f32 passes of 8 consecutive devices,
 * all passes in the same launch; results are identical to those passes and to D per-device
 * sequential mixes. Rows must be 16-byte aligned (pitch and P multiples of 4); out must not
 * overlap in. */
CFA_API int cfa_mix_ring_round_f32(float* out, const float* in, size_t pitch, const float* alphas, int D,
                                   int hl, int hr, size_t P, void* stream);

/* (f3) CFA-GE neighbour-gradient evaluation: the gradient of a device's own cost at each of M
 * neighbour models, for the two TF1 graphs of cfa_ge_2stage.py (:391-433 graph, :512-528 one
 * Session per neighbour; cfa_ge_4stage.py the same), one workgroup per model, fp32 like the
 * reference's placeholders. x [B, L] and y [B, classes] are the device's samples and one-hot
 * labels (x_train2, y_train2); models [M, P] and grads [M, P] are model buckets in the TF1
 * order (W1, b1, W2, b2), all device arrays.
 *   CNN (ML_model 1): W1 [filter, 1, number], conv stride = pool size = `stride`, SAME padding,
 *       W2 [L2 * number, classes] with L2 = ceil(ceil(L / stride) / stride) (the reference's
 *       `multip`); P = filter*number + number + L2*number*classes + classes.
 *   2NN (ML_model 2): W1 [L, hidden], W2 [hidden, classes]; P = L*hidden + hidden + hidden*classes + classes.
 * cost = mean_b(-sum_c y log(clip(softmax, 1e-15, 0.99))) (:425-426). CFA_E_UNSUPPORTED when the
 * activations of B samples do not fit one workgroup's LDS. */
CFA_API int cfa_ge_grad_cnn_f32(const float* x, const float* y, int B, int L, int classes, int filter,
                                int number, int stride, const float* models, float* grads, int M,
                                void* stream);
CFA_API int cfa_ge_grad_2nn_f32(const float* x, const float* y, int B, int L, int hidden, int classes,
                                const float* models, float* grads, int M, void* stream);
/* Population form: evaluation m uses model row model_row[m] of models [Dm, P] and data row
 * data_row[m] of x [Dx, B, L] / y [Dx, B, classes] (DEVICE int32 tables), writing grads[m]. One
 * launch evaluates every (device, neighbour) pair of a device-resident CFA-GE population: the
 * gradient of device data_row[m]'s cost at device model_row[m]'s published model. With a device
 * `workspace` of at least cfa_ge_grad_workspace_elems(M, B, P) floats, each evaluation's batch is
 * split over several workgroups (about two per CU in all) whose partial sums are then added in a
 * fixed order (deterministic); with less (or NULL) one workgroup takes each evaluation.
 * grads == NULL: partials only. The launch writes [M][S][P] partial buckets to `workspace`
 * (S = cfa_ge_grad_splits(M, B, P); at least M * S * P floats) and the caller sums them, e.g. in
 * the same launch as the next population step (cfa_ge_population_step_f32's reduce_* args). */
CFA_API int cfa_ge_grad_splits(int M, int B, size_t P);
CFA_API size_t cfa_ge_grad_workspace_elems(int M, int B, size_t P);
CFA_API int cfa_ge_grad_cnn_rows_f32(const float* x, const float* y, int B, int L, int classes,
                                     int filter, int number, int stride, const float* models,
                                     const int32_t* model_row, const int32_t* data_row, float* grads,
                                     float* workspace, size_t workspace_elems, int M, void* stream);
CFA_API int cfa_ge_grad_2nn_rows_f32(const float* x, const float* y, int B, int L, int hidden,
                                     int classes, const float* models, const int32_t* model_row,
                                     const int32_t* data_row, float* grads, float* workspace,
                                     size_t workspace_elems, int M, void* stream);

/* (a1-a6 batched) Population round: one launch mixes D devices.
 * For device d, CSR entries e in [csr_ptr[d], csr_ptr[d+1]) list its sources in order; the
 * FIRST entry is the device's own (local) bucket. Source e is src_ptrs[csr_idx[e]], output d
 * is out_ptrs[d]; both tables are DEVICE arrays of device pointers. rule:
 *   CFA_RULE_SEQUENTIAL: w = src(first); w <- w + csr_coef[e]*(src(e) - w) for later e
 *   CFA_RULE_LINEAR:     out = sum_e csr_coef[e] * src(e)
 * csr_ptr/csr_idx/csr_coef are DEVICE arrays. Outputs must not alias any source. */
CFA_API int cfa_mix_population_f32(float* const* out_ptrs, const float* const* src_ptrs,
                           const int32_t* csr_ptr, const int32_t* csr_idx,
                           const float* csr_coef, int D, int rule, size_t P, void* stream);

/* (a1/a2 batched) TF1 population round: as cfa_mix_population_f32 with the TF1 modules'
 * numerics (cfa.py:66-76 under numpy 2): per device d, w = local; the first neighbour step
 * subtracts in fp32, every later operation is fp64 with csr_coef[e] (DEVICE double array, the
 * np.float64 products eps * wf_j; entry e0's coefficient unused), and the result is rounded to
 * fp32 once: what a TF1 driver's fp32 variables hold after assigning the reference's arrays.
 * mode != CFA_COMPRESS_NONE: the cfa_ongraphs compression epilogue (cfa_ongraphs.py:225-273)
 * on elements [cbegin, cend) of every device (the W2 segment), against the device's pre-mix
 * local, before the rounding, as cfa_mix_tf1_f32 applies it; a device without neighbours gets
 * the fp32 epilogue on its local. kept_counts[d] (DEVICE, D counters, zeroed by the caller)
 * += device d's counter_param. Buckets 16-byte aligned; outputs must not alias any source. */
CFA_API int cfa_mix_population_tf1_f32(float* const* out_ptrs, const float* const* src_ptrs,
                                       const int32_t* csr_ptr, const int32_t* csr_idx,
                                       const double* csr_coef, int D, size_t P, int mode, size_t cbegin,
                                       size_t cend, unsigned long long* kept_counts, void* stream);

/* (a4 batched) CFA-GE population step: stage 1 and the gradient step of every device of a
 * device-resident population in one launch (cfa_ge_2stage.py:446-466, then :591-621). For device
 * d, CSR entries e in [csr_ptr[d], csr_ptr[d+1]): the first is its local model
 * src_ptrs[csr_idx[e0]], the others its neighbours in order, mixed with the sequential rule and
 * coefficient csr_coef[e]; then for each neighbour entry e, in order:
 *   s <- rho * g + (1 - rho) * s   (s = state_ptrs[e], g = grad_ptrs[e], NULL = zero gradient)
 *   w <- w - lr(i) * (use_filtered ? s : g),   lr(i) = i < lr_split ? lr1 : lr2
 * and out_ptrs[d] = w. Every table is a DEVICE array; entry e0's state/grad slots are unused.
 * Same operations, same order, same results as cfa_mix_population_f32 + cfa_mewma_update_f32.
 * reduce_ws != NULL: the same launch also sums the reduce_splits partial buckets of reduce_M
 * gradient evaluations (reduce_ws [reduce_M][reduce_splits][P], from a partials-only
 * cfa_ge_grad_*_rows_f32) into reduce_out [reduce_M][P], in split order: the same sums as the
 * rows launch's own reduction. A CFA-GE round is then two launches: the gradients of this round
 * (partials), and this step (previous round's gradients) + this round's reduction.
 * reduce_out must not alias any table or bucket the step reads. */
CFA_API int cfa_ge_population_step_f32(float* const* out_ptrs, const float* const* src_ptrs,
                                       float* const* state_ptrs, const float* const* grad_ptrs,
                                       const int32_t* csr_ptr, const int32_t* csr_idx,
                                       const float* csr_coef, int D, double rho, float lr1, float lr2,
                                       size_t lr_split, int use_filtered, size_t P,
                                       const float* reduce_ws, float* reduce_out, int reduce_M,
                                       int reduce_splits, void* stream);

/* ---------------------------------------------------------------------------------------
 * Multi-GPU (RCCL over xGMI): one process per GPU.
 * The reference has no collectives; its cross-device edges are files polled on a shared
 * directory (TF1/consensus/cfa.py:119-130, TF2 consensus_v3.py:82-141). When the simulated
 * population is sharded over the GPUs of one node those edges become RCCL transfers.
 */
#define CFA_UNIQUE_ID_BYTES 128

/* Fill `id` (CFA_UNIQUE_ID_BYTES bytes) on one rank; share it with the others out of band. */
/* The RCCL library version libcfa runs on (ncclGetVersion), for the record of a multi-GPU run. */
CFA_API int cfa_rccl_version(int* version);
CFA_API int cfa_comm_unique_id(void* id);
/* Create a communicator for `rank` of `nranks` on HIP device `device`. */
CFA_API int cfa_comm_init(void** comm, int rank, int nranks, const void* id, int device);
CFA_API int cfa_comm_destroy(void* comm);
/* Grouped point-to-point halo exchange of whole buckets: send_bufs[i] (P floats) goes to
 * rank send_peers[i], recv_bufs[i] is filled from recv_peers[i]. One RCCL group. */
CFA_API int cfa_halo_exchange_f32(void* comm, const float* const* send_bufs, const int* send_peers,
                          int nsend, float* const* recv_bufs, const int* recv_peers, int nrecv,
                          size_t P, void* stream);
/* Grouped point-to-point exchange of element ranges with per-message lengths: send_bufs[i]
 * (send_counts[i] floats) goes to rank send_peers[i]; recv_bufs[i] (recv_counts[i] floats) is
 * filled from recv_peers[i]. One RCCL group; messages between one rank pair pair up in issue
 * order. This is the step of the routed (multi-link, relayed) halo exchange: a group carries
 * the direct pieces and first relay hops of one stage and the second hops of the previous one
 * (federated_amd/halo.py). Zero-length messages are skipped on both sides. Replaces the same
 * file polling as cfa_halo_exchange_f32 (TF1/consensus/cfa.py:119-130). */
CFA_API int cfa_p2p_group_f32(void* comm, const float* const* send_bufs, const size_t* send_counts,
                      const int* send_peers, int nsend, float* const* recv_bufs,
                      const size_t* recv_counts, const int* recv_peers, int nrecv, void* stream);
/* Sum all-reduce / reduce of pre-scaled buckets (FedAvg / parameter-split sums). */
CFA_API int cfa_allreduce_sum_f32(void* comm, const float* send, float* recv, size_t count,
                          void* stream);
CFA_API int cfa_reduce_sum_f32(void* comm, const float* send, float* recv, size_t count, int root,
                       void* stream);

/* ---------------------------------------------------------------------------------------
 * (f2) Host-resident buckets without staging copies. Device address of a pinned host buffer
 * (hipHostMalloc, torch pin_memory). Passing it to the mix entry points makes the kernel read
 * its buckets over PCIe and write the result straight into host memory: no H2D/D2H staging,
 * and the link's two directions are busy at once. Replaces the staging copies around the mix
 * when buckets arrive in host memory: TF1/consensus/cfa.py:108-117 (.mat loads),
 * TF2 FL_threads_CIFAR100.py:424-428 (.npy), FL_over_MQTT/learner_consensus.py:136-145.
 * Fails (CFA_E_HIP) for memory the runtime has not mapped for the device.
 */
CFA_API int cfa_host_device_pointer(const void* host, void** dev);

/* ---------------------------------------------------------------------------------------
 * (f2) MQTT model payloads, host side. FL_over_MQTT ships models as
 *   pickle.dumps({'model_layer{k}': w_k.tolist(), 'device': i, 'framecount': f,
 *                 'local_epoch': e, 'training_end': b})
 * (TF2/FL_over_MQTT/learner_consensus.py:257-268; PS_server.py:137-149 answers with
 * 'global_model_layer{k}', 'global_epoch', 'training_end') and decodes them with
 * pickle.loads + np.asarray (learner_consensus.py:136-144, PS_server.py:90-118).
 * The codec below reads and writes those bytes without Python objects:
 *   - decode: one structure pass over the payload, then the float runs of a key are
 *     byte-swapped straight into a caller buffer (e.g. a pinned staging bucket), threaded for
 *     large tensors. Values equal np.asarray(pickle.loads(payload)[key]) bit for bit (fp64), or
 *     that array cast to fp32 (`_f32`). Only dict/list/str/int/bool/float/None and memo opcodes
 *     are accepted; object-constructing opcodes (GLOBAL, REDUCE, BUILD, ...) are refused, so a
 *     payload executes nothing. `buf` must stay alive and unchanged until cfa_payload_free.
 *   - encode: the exact bytes of pickle.dumps(d, protocol) (CPython 3.10, framing included)
 *     for d = {key: ndarray.tolist() | int | bool | float | None} in item order.
 */
typedef struct cfa_payload cfa_payload_t;  /* opaque parsed payload */
#define CFA_PAYLOAD_MAX_DIM 8
enum {
  CFA_PAYLOAD_NONE = 0,
  CFA_PAYLOAD_BOOL = 1,
  CFA_PAYLOAD_INT = 2,
  CFA_PAYLOAD_FLOAT = 3,
  CFA_PAYLOAD_F32_ARRAY = 4,   /* encode only: float32 data, tolist() values */
  CFA_PAYLOAD_F64_ARRAY = 5,   /* (nested) list whose np.asarray dtype is float64 */
  CFA_PAYLOAD_I64_ARRAY = 6,   /* decode only: list of ints (np.asarray -> int64) */
  CFA_PAYLOAD_BOOL_ARRAY = 7,  /* decode only: list of bools */
  CFA_PAYLOAD_STR = 8,         /* decode only */
  CFA_PAYLOAD_DICT = 9         /* decode only (nested dict; not readable as an array) */
};
typedef struct {
  const char* key;       /* NUL-terminated UTF-8 */
  int kind;              /* CFA_PAYLOAD_NONE .. CFA_PAYLOAD_F64_ARRAY */
  const void* data;      /* arrays: C-contiguous host data of `shape` */
  int ndim;              /* arrays: 0 .. CFA_PAYLOAD_MAX_DIM (0 = one float, as tolist()) */
  const int64_t* shape;  /* arrays: ndim extents */
  int64_t ivalue;        /* INT / BOOL */
  double fvalue;         /* FLOAT */
} cfa_payload_item_t;

CFA_API int cfa_payload_parse(const void* buf, size_t len, cfa_payload_t** out);
CFA_API void cfa_payload_free(cfa_payload_t* payload);
/* Number of top-level keys; negative CFA_E* on error. */
CFA_API int cfa_payload_num_keys(const cfa_payload_t* payload);
/* Key `index` (insertion order) as a pointer into the payload bytes (not NUL-terminated). */
CFA_API int cfa_payload_key(const cfa_payload_t* payload, int index, const char** key, size_t* len);
/* Kind, shape (up to CFA_PAYLOAD_MAX_DIM extents) and element count of `key`'s value. */
CFA_API int cfa_payload_info(const cfa_payload_t* payload, const char* key, int* kind, int* ndim,
                             int64_t* shape, int64_t* numel);
/* A scalar value (None / bool / int / float): ivalue for bool and int, fvalue for all. */
CFA_API int cfa_payload_scalar(const cfa_payload_t* payload, const char* key, int* kind,
                               int64_t* ivalue, double* fvalue);
/* Row-major values of `key` (numel must match) into host memory. */
CFA_API int cfa_payload_read_f64(const cfa_payload_t* payload, const char* key, double* dst,
                                 int64_t numel);
CFA_API int cfa_payload_read_f32(const cfa_payload_t* payload, const char* key, float* dst,
                                 int64_t numel);
/* Encode n items with pickle protocol 2..5. dst == NULL: only *size is set (the exact length).
 * Otherwise dst must hold cap >= *size bytes (CFA_E_INVALID if not; *size is still set). */
CFA_API int cfa_payload_encode(const cfa_payload_item_t* items, int n, int protocol, void* dst,
                               size_t cap, size_t* size);

#ifdef __cplusplus
}
#endif
#endif /* CFA_ENGINE_H */
