/*
 * rmx.h -- C ABI of the MI355X-native CTR forward path (librmx.so).
 *
 * Drop-in boundary for the reference's model plugin API
 *   abstract class RecModel           yr/model/RecModel.scala:6-127
 * and for the Angel-PS pull + gather that feeds it
 *   ParRecModel.pull* / make*         yr/model/ParRecModel.scala:165-199, 270-306
 * (paths relative to /root/reference/src/main/scala/, yr/ = io/yaochi/recommendation/).
 *
 * Two levels, one library:
 *   L-A  rmx_forward():      the exact RecModel.forward(batchSize, batch, bias, weights,
 *                            embeddings, embeddingDim, mats, matSizes[, fields]) contract
 *                            on host buffers (RecModel.scala:37-63, buildParams :146-155).
 *   L-B  rmx_forward_ids():  device-resident table + device ids (replaces pull* + make*).
 *
 * Conventions: every entry point returns 0 (RMX_OK) or a negative RMX_E_* code and
 * sets a thread-local message readable with rmx_last_error().  Calls on one model
 * are synchronous on return for L-A; L-B calls are asynchronous on the given
 * stream (pass NULL for the model's own stream; rmx_stream_sync to wait).
 * No torch types: plain pointers and sizes only.
 */
#ifndef RMX_H
#define RMX_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RMX_ABI_VERSION 1

/* Status codes -- mirror the reference's failure modes. */
#define RMX_OK 0
#define RMX_E_INVALID (-1)  /* bad argument / missing params-map key (NoSuchElementException)      */
#define RMX_E_INDEX (-2)    /* COO row index >= batchSize: bnn/Scatter.scala:29-30 require(...)       */
#define RMX_E_SHAPE (-3)    /* nnz*k != B*F*k: BigDL Reshape(B, F, k) size mismatch                    */
#define RMX_E_TYPE (-4)     /* unknown model type / array missing for the RecModelType (MatchError)    */
#define RMX_E_HIP (-5)      /* HIP runtime error                                                      */
#define RMX_E_NOMEM (-6)    /* device allocation failed                                               */
#define RMX_E_MATS (-7)     /* mats length / matSizes disagree with getMatsSize                       */
#define RMX_E_COMM (-8)     /* RCCL error in the sharded-table exchange                               */

/* Model kinds: yr/model/{lr,deepfm,xdeepfm,dcn,pnn,dnn}/ */
#define RMX_MODEL_LR 0
#define RMX_MODEL_DEEPFM 1
#define RMX_MODEL_XDEEPFM 2
#define RMX_MODEL_DCN 3
#define RMX_MODEL_PNN 4
#define RMX_MODEL_DNN 5

/* RecModelType (yr/model/RecModelType.scala:5-8). */
#define RMX_BIAS_WEIGHT 0
#define RMX_BIAS_WEIGHT_EMBEDDING 1
#define RMX_BIAS_WEIGHT_EMBEDDING_MATS 2
#define RMX_BIAS_WEIGHT_EMBEDDING_MATS_FIELD 3

/* Element types of tables and model parameters. */
#define RMX_DTYPE_F32 0
#define RMX_DTYPE_BF16 1

/* Embedding-table host layouts for rmx_table_upload. */
#define RMX_LAYOUT_K_MAJOR 0   /* reference Angel PS layout: k rows x V columns (ParRecModel.scala:95-101) */
#define RMX_LAYOUT_ROW_MAJOR 1 /* V rows x k columns                                                      */

#define RMX_FORMAT_LIBSVM 0    /* "label id:value ..."          SampleParser.parseLIBSVM (SampleParser.scala:23-51) */
#define RMX_FORMAT_LIBFFM 1    /* "label field:id:value ..."    SampleParser.parseLIBFFM (SampleParser.scala:53-85) */

typedef struct rmx_ctx rmx_ctx;
typedef struct rmx_model rmx_model;
typedef struct rmx_table rmx_table;
typedef struct rmx_shard rmx_shard;
typedef struct rmx_group rmx_group;
typedef struct rmx_samples rmx_samples;

/* ------------------------------------------------------------------ misc -- */
const char* rmx_last_error(void);
int rmx_abi_version(void);

/* Process-wide tuning knobs (kernel variant selection for A/B timing in one process).
 * Known keys (README.md lists them): "f32_split", "s3_tower", "s3_dense", "s3_cin", "tower_variant" (GEMM
 * engine and tile variants, csrc/k_gemm.hpp, k_gemm_s3.hip), "fm_fuse", "fm_y1", "fo_fuse" (first
 * order / FM inside tower layer 1), "wgrad_s3" (training dW kernel, csrc/train.hip).  Unknown keys
 * are stored and ignored.  rmx_get_tuning returns def when the key was never set; setting
 * RMX_TUNING_DEFAULT removes the key (back to the built-in default). */
#define RMX_TUNING_DEFAULT (-2147483647 - 1)
int rmx_set_tuning(const char* key, int value);
int rmx_get_tuning(const char* key, int def);

/* ------------------------------------------------------------- context ---- */
/* One context per (process, GPU).  Owns a HIP stream. */
int rmx_ctx_create(int device, rmx_ctx** out);
int rmx_ctx_destroy(rmx_ctx* ctx);
void* rmx_ctx_stream(rmx_ctx* ctx);            /* hipStream_t of the context */
int rmx_stream_sync(void* stream);             /* hipStreamSynchronize        */

/* Device memory helpers for L-B callers (ids / outputs resident in HBM). */
int rmx_malloc(rmx_ctx* ctx, size_t bytes, void** dptr);
int rmx_free(rmx_ctx* ctx, void* dptr);
int rmx_memcpy_htod(rmx_ctx* ctx, void* dst, const void* src, size_t bytes);
int rmx_memcpy_dtoh(rmx_ctx* ctx, void* dst, const void* src, size_t bytes);

/* HIP events on the given stream (NULL = context stream), for in-band timing. */
int rmx_event_create(void** ev);
int rmx_event_destroy(void* ev);
int rmx_event_record(void* ev, void* stream);
int rmx_event_elapsed_ms(void* start, void* stop, float* ms);

/* ---------------------------------------------------------------- model ---- */
/* new LR(inputDim)                                       yr/model/lr/LR.scala:10
 * new DeepFM(inputDim, nFields, embeddingDim, fcDims)      yr/model/deepfm/DeepFM.scala:10
 * new XDeepFM(inputDim, nFields, embeddingDim, fcDims, cinDims)  yr/model/xdeepfm/XDeepFM.scala:10
 * new DCN(inputDim, nFields, embeddingDim, crossDepth, fcDims)   yr/model/dcn/DCN.scala:10
 * new PNN(inputDim, nFields, embeddingDim, fcDims)         yr/model/pnn/PNN.scala:10
 * new DNN(inputDim, nFields, embeddingDim, fcDims)         yr/model/dnn/DNN.scala:10
 * Unused arguments are ignored (pass 0 / NULL).  ctx may be NULL for a host-only model that
 * answers the metadata calls (getMatsSize ...) without a GPU. */
int rmx_model_create(rmx_ctx* ctx, int type, int64_t input_dim, int n_fields, int embedding_dim,
                     const int32_t* fc_dims, int n_fc, const int32_t* cin_dims, int n_cin,
                     int cross_depth, rmx_model** out);
int rmx_model_destroy(rmx_model* m);
/* RecModel.getType / getMatsSize / getInputDim / getEmbeddingDim (RecModel.scala:7, :121-125).
 * getMatsSize writes up to cap ints into sizes and stores the full count in *n. */
int rmx_model_get_type(const rmx_model* m);
int rmx_model_get_mats_size(const rmx_model* m, int32_t* sizes, int cap, int* n);
int64_t rmx_model_mats_len(const rmx_model* m);
int64_t rmx_model_get_input_dim(const rmx_model* m);
int rmx_model_get_embedding_dim(const rmx_model* m);

/* L-A: RecModel.forward(batchSize, batch: CooLongFloatMatrix, bias, weights, embeddings,
 *        embeddingDim, mats, matSizes[, fields]): Array[Float]     RecModel.scala:9-63
 * index[nnz] = batch.getRowIndices, feats[nnz] = batch.getColIndices (unused by the math,
 * as in the reference), weights[nnz] / embedding[nnz*k] already gathered by the caller,
 * bias[1].  Arrays not used by the model's RecModelType may be NULL.  fields is ignored
 * (no reference model reads it).  out[batch_size] receives sigmoid probabilities. */
int rmx_forward(rmx_model* m, int32_t batch_size, int64_t nnz, const int64_t* index,
                const int64_t* feats, const float* bias, const float* weights,
                const float* embedding, int32_t embedding_dim, const float* mats,
                const int32_t* mat_sizes, int32_t n_sizes, const int64_t* fields, float* out);

/* L-A backward: RecModel.backward(batchSize, batch, bias, weights, embeddings, embeddingDim,
 *        mats, matSizes[, fields], targets): Float                RecModel.scala:65-115
 * Same arrays and checks as rmx_forward plus targets[batch_size] (label > 0 -> 1).  On return the
 * caller's bias / weights / embedding / mats arrays hold the GRADIENTS, as the reference writes
 * them back in place (yr/util/GradUtil.scala:7-42, BackwardUtil.scala:6-30), and *loss the mean
 * BCE loss (BigDL BCECriterion, sizeAverage).  fp32 models; every model kind (LR, DeepFM, xDeepFM,
 * DCN, PNN, DNN). */
int rmx_backward(rmx_model* m, int32_t batch_size, int64_t nnz, const int64_t* index,
                 const int64_t* feats, float* bias, float* weights, float* embedding,
                 int32_t embedding_dim, float* mats, const int32_t* mat_sizes, int32_t n_sizes,
                 const int64_t* fields, const float* targets, float* loss);

/* Deterministic synthetic mats (Xavier-uniform weights, U(-0.01, 0.01) biases), bit-identical
 * to oracle/orc_init_mats; works on host-only models (ctx == NULL). */
int rmx_model_init_mats(const rmx_model* m, uint64_t seed, float* mats);

/* L-B parameters: load mats (getMatsSize layout) and the global bias once, on device. */
int rmx_model_set_mats(rmx_model* m, const float* mats, int64_t n_mats);
int rmx_model_set_bias(rmx_model* m, float bias);
/* RMX_DTYPE_BF16: Linear weights stored bf16 (rounded to nearest even when mats are loaded), the
 * towers on bf16 MFMA with fp32 accumulation, stored activations bf16 (BASELINE.json configs[4]).
 * Biases, the output Linear and DCN cross vectors stay fp32.  Call before rmx_model_set_mats.
 * L-B needs a table of the same dtype; L-A rounds the caller's fp32 arrays.  Not for xDeepFM. */
int rmx_model_set_precision(rmx_model* m, int dtype);

/* ---------------------------------------------------------------- table ---- */
/* HBM-resident first-order weights + embedding table (replaces the Angel PS rows
 * "weights" and "embedding", ParRecModel.scala:74-105).  Stored row-major [V][k]. */
int rmx_table_create(rmx_ctx* ctx, int64_t num_rows, int embedding_dim, rmx_table** out);
/* dtype RMX_DTYPE_BF16: the table stores bf16 (BASELINE.json configs[4]); uploads and the
 * synthetic fill round fp32 values to nearest even. */
int rmx_table_create_ex(rmx_ctx* ctx, int64_t num_rows, int embedding_dim, int dtype, rmx_table** out);
int rmx_table_dtype(const rmx_table* t);
int rmx_table_destroy(rmx_table* t);
/* Host upload; weights may be NULL, embedding may be NULL (then left as is). */
int rmx_table_upload(rmx_table* t, const float* weights, const float* embedding, int layout);
/* Deterministic synthetic fill, bit-identical to oracle/orc_gen_table (U(-0.05, 0.05)). */
int rmx_table_fill_synthetic(rmx_table* t, uint64_t seed);
int64_t rmx_table_rows(const rmx_table* t);
int rmx_table_embedding_dim(const rmx_table* t);  /* k of the table (-1: NULL) */
/* With knob "table_lines" 1 (default 0), fp32 k = 16 tables also hold a [rows][32] line copy
 * ([emb 16 | w | pad]: one 128-B memory line per id) that DeepFM / DNN / LR forwards read; every
 * upload / fill rebuilds it.  After writing the table through rmx_table_device_ptrs, call
 * rmx_table_refresh_lines (it also builds or drops the copy after the knob changes). */
int rmx_table_refresh_lines(rmx_table* t);
/* Device pointers of the table (for debugging/parity only; elements of the table's dtype). */
int rmx_table_device_ptrs(const rmx_table* t, void** d_weights, void** d_embedding);

/* Synthetic field-partitioned ids into device memory, bit-identical to orc_gen_ids. */
int rmx_gen_ids(rmx_ctx* ctx, uint64_t seed, int64_t row0, int32_t batch, int32_t n_fields,
                int64_t num_rows, int32_t* d_ids, void* stream);
/* L-B backward on the device-resident table: one training pass (forward with stored
 * activations, BCE, gradients) over ids [B][F].  Device outputs, each may be NULL: g_bias[1],
 * g_weights[B*F] (per nonzero, Scatter backward), g_embedding[B*F*k] (per nonzero),
 * g_mats[mats_len] (getMatsSize layout), loss[1].  The sparse per-nonzero gradients are what the
 * reference hands to makeGrad/push (ParRecModel.scala:439-478). */
int rmx_backward_ids(rmx_model* m, const rmx_table* t, int32_t batch, const int32_t* d_ids,
                     const float* d_targets, float* d_g_bias, float* d_g_weights, float* d_g_embedding,
                     float* d_g_mats, float* d_loss, void* stream);

/* Predict loop over a device-resident row set (ParRecModel.predict*, ParRecModel.scala:519-581):
 * scores[r] for rows r < n_rows of ids [n_rows][F], forwards of `batch` rows. */
int rmx_predict_ids(rmx_model* m, const rmx_table* t, int64_t n_rows, const int32_t* d_ids,
                    int32_t batch, float* d_scores, void* stream);
/* AUC of (label > 0, score) pairs on the device (the examples' per-epoch metric,
 * example/DeepFMLocalExample.scala:44-52): Mann-Whitney statistic, tied scores count 1/2.
 * *auc = NaN when one class is empty.  Synchronises the stream. */
int rmx_auc(rmx_ctx* ctx, int64_t n, const float* d_labels, const float* d_scores, double* auc,
            void* stream);

/* Zipf-like ids (SURVEY.md §8d secondary): rank r of field f drawn with P(r) ~ (r+1)^-exponent
 * (continuous power-law inversion, double precision), id = f * (num_rows / n_fields) + r. */
int rmx_gen_ids_zipf(rmx_ctx* ctx, uint64_t seed, int64_t row0, int32_t batch, int32_t n_fields,
                     int64_t num_rows, double exponent, int32_t* d_ids, void* stream);

/* Test hook: fill the LDS of every CU with a 32-bit pattern (e.g. 0x7FC00000, a NaN) on the stream, so a
 * kernel launched next that reads LDS it never wrote reads that pattern (tests/test_small_s3.py). */
int rmx_debug_fill_lds(rmx_ctx* ctx, uint32_t pattern, void* stream);

/* Test hook (host only, no GPU): the slice count S the training dW on the 208 x 208 tile uses for a
 * rows x N x K weight gradient on a device with ncu CUs.  S fixes the dW's fp32 summation order over the
 * slices, so gradients are bitwise reproducible across devices with the same CU count (every 256-CU
 * MI355X), not across CU counts.  Returns S (> 0) or RMX_E_INVALID. */
int rmx_debug_wgrad_slices(int64_t rows, int N, int K, int ncu);

/* Debug gather: d_w[n] = weights[ids[n]], d_emb[n*k+j] = emb[ids[n]][j] (makeWeights /
 * makeEmbeddings, ParRecModel.scala:279-306).  Bit-exact copies (as fp32 for a bf16 table). */
int rmx_gather(const rmx_table* t, int64_t n, const int32_t* d_ids, float* d_w, float* d_emb,
               void* stream);

/* L-B forward: d_ids[batch * nFields] (int32, device), d_out[batch] (device).
 * Requires rmx_model_set_mats / rmx_model_set_bias first.  Asynchronous on stream. */
int rmx_forward_ids(rmx_model* m, const rmx_table* t, int32_t batch, const int32_t* d_ids,
                    float* d_out, void* stream);

/* Per-stage timing of the last rmx_forward_ids calls made with timing enabled:
 * names/ms of up to cap stages (kernels) accumulated since enable. */
int rmx_model_set_timing(rmx_model* m, int enable);
int rmx_model_get_timing(rmx_model* m, char* names, int name_stride, float* ms, int cap, int* n,
                         int* calls);

/* Encoder-only launch (gather + first order + FM for DeepFM, first order otherwise):
 * d_y[batch] = y1 + y2 (DeepFM) / y1.  Used to measure the HBM-bound encoder alone. */
int rmx_encoder_ids(rmx_model* m, const rmx_table* t, int32_t batch, const int32_t* d_ids,
                    float* d_y, void* stream);

/* -------------------------------------------------------- sharded table ---- */
/* Hash-sharded table over nranks processes, one GPU each (BASELINE.json configs[3]): replaces
 * the column-range-partitioned Angel PS matrices and their sparse pulls (ParRecModel.scala:74-105,
 * :165-199).  owner(id) = p(id) mod nranks, local row = p(id) div nranks, p the keyed permutation of
 * rmx_shard_set_owner_hash (default key RMX_OWNER_HASH_DEFAULT).  One exchange per batch over
 * RCCL (grouped send/recv = all-to-all over xGMI): ids to owners, rows back.
 * At nranks > 1 the exchange has fixed-capacity buckets (~1.1 x ids / nranks per peer): every message
 * size is known on the host, so the exchange makes no host sync; ids past a bucket's capacity get their
 * rows in a second, counted round that every rank runs when any rank overflowed (each rank's header
 * carries its overflow flag).  The overflow check is made when the slot is consumed (or, for
 * rmx_forward_ids_sharded / rmx_shard_gather, after the forward / copy is queued, which then runs again).
 * An id outside [0, num_rows) reads a zero row on every path.
 * An exchange that fails on a rank at nranks > 1 (e.g. out of device memory while routing) leaves that
 * rank's collectives out of step with its peers': every later exchange on the shard returns RMX_E_COMM at
 * once.  Abort the shard on every rank (rmx_shard_abort, then rmx_shard_destroy) and create a new one;
 * peers already waiting in the failed exchange are released by their own abort (e.g. a watchdog).
 * The first exchange of a shard has no agreed bucket capacity yet, so all of its ids take the counted
 * overflow round (one extra round, once; timed under the "shard_exchange" stage) -- unless every rank
 * called rmx_shard_set_batch_hint with the same ids-per-batch figure first, which seeds that capacity.
 * CONTRACT CHANGE (round 3): the default owner function is the keyed permutation below, no longer
 * id mod nranks.  A caller that pre-partitions ids or rows must use rmx_owner_hash (or
 * rmx_shard_set_owner_hash(sh, 0) for id mod nranks). 
 * rmx_comm_unique_id: rank 0 creates the RCCL id (RMX_UNIQUE_ID_BYTES bytes) and the caller
 * broadcasts it (e.g. torch.distributed / MPI / Spark broadcast).  unique_id == NULL creates a
 * LOOPBACK shard: all nranks partitions live in this process on ctx's GPU and the exchange is
 * in-device (single-GPU testing of the routing at nranks > 1). */
#define RMX_UNIQUE_ID_BYTES 128
int rmx_comm_unique_id(void* out, size_t cap);
int rmx_shard_create(rmx_ctx* ctx, int64_t num_rows, int embedding_dim, int nranks, int rank,
                     const void* unique_id, rmx_shard** out);
int rmx_shard_destroy(rmx_shard* sh);
/* Abort the shard's RCCL communicator (ncclCommAbort) from any thread, e.g. a watchdog while an
 * exchange waits for a peer that never arrives: the pending exchange fails (or its kernels return)
 * and every later exchange returns RMX_E_COMM; only rmx_shard_destroy may follow.  Waits (at most 5 s)
 * for an exchange's host-side RCCL calls in flight on another thread to finish first, so no ncclSend /
 * ncclGroupEnd runs on the communicator while it is torn down.  A no-op returning RMX_OK for loopback and group shards. */
int rmx_shard_abort(rmx_shard* sh);
/* Owned rows from the same generator as rmx_table_fill_synthetic (bit-identical rows). */
int rmx_shard_fill_synthetic(rmx_shard* sh, uint64_t seed);
int64_t rmx_shard_local_rows(const rmx_shard* sh);
/* Owner function (before rmx_shard_fill_synthetic; every rank the same key): owner = p(id) mod
 * nranks, local row = p(id) div nranks with p a keyed pseudo-random permutation of [0, num_rows)
 * (4-round Feistel, cycle-walked), so strided or clustered id spaces spread evenly (the table is
 * HASH-sharded by default: key RMX_OWNER_HASH_DEFAULT); key 0 = the identity, owner = id mod nranks.
 * rmx_shard_owner_of: the rank owning id (-1 if out of range).  rmx_owner_hash: the same function
 * without a shard (host only): the owner of id, *local_row (nullable) its row there; -1 if id is
 * outside [0, num_rows) or the arguments are bad. */
#define RMX_OWNER_HASH_DEFAULT 0x5EED5A4D0C7A11EDULL
int rmx_shard_set_owner_hash(rmx_shard* sh, uint64_t key);
int64_t rmx_shard_owner_of(const rmx_shard* sh, int64_t id);
int64_t rmx_owner_hash(uint64_t key, int64_t num_rows, int nranks, int64_t id, int64_t* local_row);
/* Step 0 of the exchange: send each DISTINCT id of the batch once, as
 * ParRecModel.distinctIntIndices (ParRecModel.scala:337-345) before the pull; results are identical.
 * on: 0 off, 1 on, 2 auto (default: off at one rank; else on for a batch, then off for the next 63
 * batches when it removed fewer than 10 % of the ids, re-probed after them). */
int rmx_shard_set_dedupe(rmx_shard* sh, int on);
/* Seeds the first fixed-capacity exchange's bucket capacity from nnz, the ids one rank sends per batch
 * (B * nFields; the reference's batchSize * fields, ParRecModel.scala:165-199): ~1.1 nnz / nranks per
 * peer.  Collective by value: every rank must pass the same nnz before its first exchange.  Later
 * exchanges size their buckets from the previous one as before.  Without it the first exchange runs its
 * ids through the counted overflow round. */
int rmx_shard_set_batch_hint(rmx_shard* sh, int64_t nnz);
/* Ids this rank sent to owners in its last exchange (the distinct ids when deduplicating). */
int64_t rmx_shard_last_sent(const rmx_shard* sh);
/* Overflow rounds this shard has run (fixed-capacity exchange at nranks > 1: an id past its bucket's
 * capacity on any rank); -1 for a NULL shard. */
int64_t rmx_shard_overflow_rounds(const rmx_shard* sh);
/* Collective (every rank calls it): d_w[i] = w[ids[i]], d_emb[i*k+j] = emb[ids[i]][j] gathered
 * from the owners (makeWeights / makeEmbeddings through the exchange).  Bit-exact copies. */
int rmx_shard_gather(rmx_shard* sh, int64_t n, const int32_t* d_ids, float* d_w, float* d_emb,
                     void* stream);
/* In-process exchange group: nranks VIRTUAL ranks in one process (one host thread, context and
 * stream each, all on one GPU or several).  A shard created on a group runs the same exchange
 * schedule as the RCCL one (counts, ids to owners, owner gather, rows back, own bucket local), with
 * every grouped send/recv replaced by a device copy from the peer's posted buffer; the ranks
 * rendezvous inside each grouped step, so every rank must make the same collective calls, each from
 * its own thread (a rank missing for 120 s fails the step with RMX_E_COMM).  Used to run the
 * N > 1 exchange on a single GPU.  The group lives until it and all its shards are destroyed. */
int rmx_group_create(int nranks, rmx_group** out);
int rmx_group_destroy(rmx_group* g);
int rmx_shard_create_group(rmx_ctx* ctx, int64_t num_rows, int embedding_dim, rmx_group* group, int rank,
                           rmx_shard** out);
/* Collective: L-B forward of this rank's batch (d_ids [batch * nFields]) over the sharded table
 * (exchange + forward on one stream, through pull slot 0). */
int rmx_forward_ids_sharded(rmx_model* m, rmx_shard* sh, int32_t batch, const int32_t* d_ids,
                            float* d_out, void* stream);
/* The same split in two, so batch i + 1's exchange overlaps batch i's forward (the reference's pull*
 * then forward, ParRecModel.scala:165-199 / :279-306):
 *   rmx_shard_pull     (collective) exchange n ids into pull slot 0 or 1 on `stream`;
 *   rmx_forward_pulled forward of the batch in that slot on `stream` (typically another stream: it
 *                      waits for the pull on the device, and the slot's next pull waits for it).
 * A slot holds one pull until its forward consumes it (a second pull into it fails RMX_E_INVALID). */
int rmx_shard_pull(rmx_shard* sh, int64_t n, const int32_t* d_ids, int slot, void* stream);
int rmx_forward_pulled(rmx_model* m, rmx_shard* sh, int32_t batch, int slot, float* d_out, void* stream);

/* ---- samples: native LIBSVM / LIBFFM parser (host, multi-threaded) ----
 * Replaces SampleParser.parse (yr/data/SampleParser.scala:14-85) for text in memory (one sample per
 * '\n'-terminated line): rows[nnz] = line index, cols[nnz] = id - 1, values[nnz], targets[lines] =
 * labels, fields[nnz] (LIBFFM only).  Malformed lines fail with RMX_E_INVALID naming the line, where
 * the reference throws NumberFormatException / ArrayIndexOutOfBoundsException.  nthreads <= 0:
 * all hardware threads.  The arrays stay valid until rmx_samples_free. */
int rmx_samples_parse(const char* text, size_t len, int format, int nthreads, rmx_samples** out);
int rmx_samples_free(rmx_samples* s);
int64_t rmx_samples_lines(const rmx_samples* s);
int64_t rmx_samples_nnz(const rmx_samples* s);
const int64_t* rmx_samples_rows(const rmx_samples* s);
const int64_t* rmx_samples_cols(const rmx_samples* s);
const float* rmx_samples_values(const rmx_samples* s);
const float* rmx_samples_targets(const rmx_samples* s);
const int64_t* rmx_samples_fields(const rmx_samples* s);  /* NULL for LIBSVM */
/* ids [lines][n_fields] (int32, ParRecModel.scala:342 .toInt) of a regular batch (every line has
 * exactly n_fields pairs: the models' Reshape(B, F, k)); RMX_E_SHAPE otherwise. */
int rmx_samples_ids(const rmx_samples* s, int32_t n_fields, int32_t* ids, int64_t cap);

#ifdef __cplusplus
}
#endif
#endif
