/*
 * stc.h — the C ABI of libstc.so, the MI355X-native text-clustering hot path.
 *
 * This is the drop-in boundary: the entry points a JNI shim binds so that
 * the reference's Spark pipeline can route its hot path to HIP kernels on gfx950.  Plain C
 * types only (pointers + sizes); no torch, no C++ in the signatures.
 *
 * Which reference interface each entry point replaces ([U] = upstream spark-mllib 2.4.3,
 * TextClustering/build.sbt:10; paths relative to /root/reference/TextClustering/src/main/scala):
 *
 *   stc_tokenize[_hashing_tf_dev] [U] ml.feature.Tokenizer (toLowerCase.split("\\s")), the step in
 *                               front of HashingTF (the reference's own
 *                               CoreNLP front-end at LDAClustering.scala:116-139 is out of scope)
 *   stc_hashing_tf[_dev]        [U] mllib.feature.HashingTF.transform / murmur3Hash — the slot of
 *                               the vocab-indexed counting at LDAClustering.scala:154-167
 *   stc_idf_fit                 IDF(minDocFreq).fit(tf).idf — LDAClustering.scala:177
 *   stc_idf_transform           tf × idf (+ the 0 → 1e-4 floor) — LDAClustering.scala:180-192
 *   stc_lda_create / set_corpus new LDA().setOptimizer(online)...setK... — LDAClustering.scala:37-54
 *                               ([U] OnlineLDAOptimizer.initialize)
 *   stc_lda_next / stc_lda_step one OnlineLDAOptimizer.next() / submitMiniBatch inside
 *                               lda.run(corpus) — LDAClustering.scala:61
 *   stc_lda_get_topics          [U] LocalLDAModel.topicsMatrix (getLDAModel)
 *   stc_lda_describe            ldaModel.describeTopics(maxTermsPerTopic) — LDAClustering.scala:81,
 *                               LDALoader.scala:66
 *   stc_lda_topic_distribution  toLocal.topicDistribution(tf) — LDALoader.scala:108
 *   stc_lda_bound               [U] LocalLDAModel.logLikelihood / logPerplexity
 *   stc_comm_*                  the role of Spark's broadcast + treeReduce inside lda.run
 *                               (per minibatch: RCCL reduce-scatter of the k×V sstats over
 *                               vocabulary slices, the slice's λ update, all-gather of expElogβ)
 *
 * Conventions
 *   - Every function returns STC_OK (0) or an STC_ERR_* code; the message of the last failure on
 *     the calling thread is returned by stc_last_error().  The library never aborts.
 *   - The caller owns every host array; output arrays are caller-allocated with the sizes given
 *     in each comment.  The library owns all device memory behind the opaque handles.
 *   - A handle is not thread-safe: serialise calls per handle.  One stc_ctx = one GPU.  Several
 *     GPUs are driven either from ONE process through an stc_group (one handle, N devices, one
 *     host thread per member inside each group call — the JVM drop-in's form, Spark local[*]), or
 *     by one process per GPU whose contexts are connected with stc_comm_init.
 *   - Matrices are row-major.  The topics matrix crosses the boundary as V×k (Spark's
 *     topicsMatrix orientation, element (v, t) at [v*k + t]) unless a KV layout flag is given.
 */
#ifndef STC_H_
#define STC_H_

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STC_ABI_VERSION 2  /* 2: stc_lda_config.mixed_resolve_iters, STC_MIXED */

enum stc_status {
  STC_OK = 0,
  STC_ERR_INVALID_ARG = 1, /* maps to IllegalArgumentException on the JVM side */
  STC_ERR_HIP = 2,         /* HIP runtime error (IllegalStateException) */
  STC_ERR_RCCL = 3,        /* RCCL error */
  STC_ERR_OOM = 4,         /* device allocation failed */
  STC_ERR_STATE = 5        /* call not valid in the handle's current state */
};

/* The reference pins spark-mllib 2.4.3 (TextClustering/build.sbt:10), whose HashingTF hashes with the
 * legacy tail: callers reproducing the reference's pipeline pass STC_HASH_SPARK24 (the Python mirror's
 * default, stc.HashingTF(hashAlgorithm="murmur3-spark24")).  The two agree iff len % 4 == 0. */
enum stc_hash_variant {
  STC_HASH_STANDARD = 0, /* MurmurHash3_x86_32 (Spark 3.x hashUnsafeBytes2) */
  STC_HASH_SPARK24 = 1   /* Spark 2.4.x hashUnsafeBytes: per-byte sign-extended tail */
};

enum stc_dtype {
  STC_F32 = 0,
  STC_F64 = 1,
  /* an LDA dtype only (stc_lda_config.dtype; the corpus CSR is STC_F64): the fp32 E-step for every document,
   * then the documents whose fp32 fixed point took more than mixed_resolve_iters iterations — the slowly
   * contracting ones, where fp32 rounding moves the stopping iterate — re-solved from the same γ₀ in fp64
   * (expElogβ' kept in both precisions); sstats, stat and the expElogβ' the E-step reads in fp32, λ / α /
   * colsum / the bound in fp64.  Inference (bound, topicDistribution) runs in fp64. */
  STC_MIXED = 2
};

enum stc_layout {
  STC_LAYOUT_VK = 0, /* V×k row-major: topicsMatrix(v, t) at [v*k + t] */
  STC_LAYOUT_KV = 1  /* k×V row-major: Spark's internal λ / a column-major topicsMatrix */
};

typedef struct stc_ctx stc_ctx;   /* one device (+ optional RCCL communicator) */
typedef struct stc_dcsr stc_dcsr; /* device-resident CSR matrix (rows = documents) */
typedef struct stc_lda stc_lda;   /* online-LDA optimizer state / LocalLDAModel */

/* ---- library / device ------------------------------------------------------------------ */
const char* stc_last_error(void);
int stc_abi_version(void);
int stc_device_count(int* n_out);
int stc_init(int device, stc_ctx** out);
int stc_destroy(stc_ctx* ctx);
int stc_synchronize(stc_ctx* ctx);

/* ---- RCCL: one process per GPU ---------------------------------------------------------
 * Rank 0 calls stc_comm_unique_id and ships the 128 bytes to the other ranks out of band
 * (the Spark driver broadcast, or torch.distributed's store); every rank then calls
 * stc_comm_init.  Once connected, stc_idf_fit, stc_lda_step/next and stc_lda_bound reduce
 * their partial results over all ranks (RCCL over xGMI), and the M-step is sharded: each rank
 * updates λ on its vocabulary slice, so the λ readers stc_lda_get_topics / stc_lda_describe
 * become collective too (every rank calls them; the first after a step all-gathers λ).
 * Connect before stc_lda_create (a later connect re-lays the model out before the next step). */
int stc_comm_unique_id(uint8_t id_out[128]);
int stc_comm_init(stc_ctx* ctx, const uint8_t id[128], int n_ranks, int rank);
int stc_comm_allreduce_f64(stc_ctx* ctx, double* host_inout, int64_t n); /* host scalars */

/* ---- device CSR ------------------------------------------------------------------------- */
/* values are stored on device as `value_dtype` (STC_F32 or STC_F64).  A device object (stc_dcsr,
 * stc_dtok) belongs to the stc_ctx that made it: every call that reads it requires that same ctx (or an
 * LDA handle created on it) and returns STC_ERR_INVALID_ARG otherwise.  The *_free calls remember the
 * device, not the ctx, so they remain valid after stc_destroy of the owning context. */
int stc_dcsr_upload(stc_ctx* ctx, int64_t n_rows, int64_t n_cols, const int64_t* indptr,
                    const int32_t* indices, const double* values, int value_dtype,
                    stc_dcsr** out);
int stc_dcsr_shape(const stc_dcsr* m, int64_t* n_rows, int64_t* n_cols, int64_t* nnz);
/* indptr[n_rows+1], indices[nnz], values[nnz] (any may be NULL to skip) */
int stc_dcsr_download(stc_ctx* ctx, const stc_dcsr* m, int64_t* indptr, int32_t* indices,
                      double* values);
/* Waits for the device to finish queued work, then hands the buffers back to the owning context for
 * reuse.  Detach a training corpus from every stc_lda (stc_lda_set_corpus with another matrix, or
 * stc_lda_destroy) before freeing it: the handle keeps a reference. */
int stc_dcsr_free(stc_dcsr* m);

/* ---- HashingTF (K1 murmur3 + nonNegativeMod, K2 per-doc count → sorted CSR) -----------
 * Tokens are given as one UTF-8 byte blob: token t is utf8[tok_off[t] .. tok_off[t+1]),
 * document d owns tokens [doc_off[d], doc_off[d+1]).  Output row d holds the sorted distinct
 * bucket indices nonNegativeMod(murmur3_x86_32(token, seed 42), num_features) and their
 * counts (1.0 when binary).  Bit-exact with [U] HashingTF.transform.                      */
int stc_hashing_tf_dev(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes,
                       const int64_t* tok_off /* n_tok+1 */, int64_t n_tok,
                       const int64_t* doc_off /* n_docs+1 */, int64_t n_docs,
                       int32_t num_features, int binary, int hash_variant, int value_dtype,
                       stc_dcsr** out);
/* host-in/host-out convenience: indices_out/values_out need capacity n_tok */
int stc_hashing_tf(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                   int64_t n_tok, const int64_t* doc_off, int64_t n_docs, int32_t num_features,
                   int binary, int hash_variant, int64_t* indptr_out /* n_docs+1 */,
                   int32_t* indices_out, double* values_out);
/* device-resident token input: the same (utf8, tok_off, doc_off) triple uploaded once, for callers that
 * keep the corpus on the GPU between calls (and for timing the kernels without the PCIe upload) */
typedef struct stc_dtok stc_dtok;
int stc_tokens_upload(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                      int64_t n_tok, const int64_t* doc_off, int64_t n_docs, stc_dtok** out);
int stc_tokens_free(stc_dtok* t);
int stc_hashing_tf_tokens(stc_ctx* ctx, const stc_dtok* tokens, int32_t num_features, int binary,
                          int hash_variant, int value_dtype, stc_dcsr** out);
/* raw per-token bucket indices (test hook for K1): idx_out[n_tok] */
int stc_hash_tokens(stc_ctx* ctx, const uint8_t* utf8, int64_t n_bytes, const int64_t* tok_off,
                    int64_t n_tok, int32_t num_features, int hash_variant, int32_t* idx_out);

/* ---- Tokenizer (K0) ----------------------------------------------------------------------
 * Document d is the UTF-8 string text[text_off[d] .. text_off[d+1]).  Output: Spark's
 * Tokenizer result — lower-case, split on each Java \\s character ([ \t\n\x0B\f\r]), interior empty
 * tokens kept, trailing empty tokens dropped, a separator-free string is one token ("" → [""]) —
 * laid out as stc_hashing_tf's input: the separator-free lower-cased blob utf8_out (utf8_cap bytes;
 * n_bytes + n_bytes / 2 always suffices: lower-casing can grow a 2-byte character to 3 bytes — when the
 * text needs more than utf8_cap the call fails with STC_ERR_INVALID_ARG before writing any output and
 * *n_out_bytes holds the size needed), tok_off_out (capacity n_bytes + n_docs + 1) and doc_off_out[n_docs+1].
 * Size query: utf8_out = NULL with utf8_cap = 0 returns STC_OK with only *n_out_bytes (and *n_tok_out when
 * given) set; tok_off_out and doc_off_out may then be NULL.
 * Lower-casing is Java 8's String.toLowerCase (root locale, Unicode 6.2) for every code point: the BMP
 * through a generated table, Deseret inline, characters Java 8 does not case passed through, and the 18
 * code points whose mapping is not a same-length 1:1 map by rule: U+0130 İ → "i̇" (2 → 3 bytes), U+03A3 Σ
 * → ς / σ by its Final_Sigma context, and the capitals whose lower case changes UTF-8 length (U+023A,
 * U+023E, U+1E9E, U+2126, U+212A, U+212B, U+2C62, U+2C64, U+2C6D–U+2C70, U+2C7E, U+2C7F, U+A78D, U+A7AA). */
int stc_tokenize(stc_ctx* ctx, const uint8_t* text, int64_t n_bytes, const int64_t* text_off,
                 int64_t n_docs, uint8_t* utf8_out, int64_t utf8_cap, int64_t* n_out_bytes,
                 int64_t* tok_off_out, int64_t* n_tok_out, int64_t* doc_off_out);
/* Tokenizer → HashingTF fused on device (no host round trip between the two stages) */
int stc_tokenize_hashing_tf_dev(stc_ctx* ctx, const uint8_t* text, int64_t n_bytes,
                                const int64_t* text_off, int64_t n_docs, int32_t num_features,
                                int binary, int hash_variant, int value_dtype, stc_dcsr** out);

/* ---- IDF (K3 df count, K4 idf, K5 transform) ---------------------------------------------
 * df_j = #rows with value_j > 0, m = #rows (summed over all ranks when connected);
 * idf_j = df_j >= min_doc_freq ? ln((m+1)/(df_j+1)) : 0.                                  */
int stc_idf_fit(stc_ctx* ctx, const stc_dcsr* tf, int64_t min_doc_freq,
                double* idf_out /* n_cols */, int64_t* df_out /* n_cols, may be NULL */,
                int64_t* m_out /* may be NULL */);
/* values[e] *= idf[indices[e]]; when zero_floor > 0 an idf of exactly 0 is replaced by
 * zero_floor (the reference's LDAClustering.scala:184-187 quirk; 0 = stock Spark)          */
int stc_idf_transform(stc_ctx* ctx, stc_dcsr* tf, const double* idf /* n_cols */,
                      double zero_floor);
/* The same IDFModel kept on the device (the GPU-resident HashingTF → IDF → LDA pipeline: the idf
 * vector need not cross PCIe between fit and transform); stc_idf_get copies it out (any may be NULL). */
typedef struct stc_didf stc_didf;
int stc_idf_fit_dev(stc_ctx* ctx, const stc_dcsr* tf, int64_t min_doc_freq, stc_didf** out);
int stc_idf_get(stc_ctx* ctx, const stc_didf* model, double* idf_out /* n_cols */,
                int64_t* df_out /* n_cols */, int64_t* m_out);
int stc_idf_transform_dev(stc_ctx* ctx, stc_dcsr* tf, const stc_didf* model, double zero_floor);
/* the model's vector size (numFeatures: stc_idf_get writes n_cols values to each output) and m */
int stc_didf_shape(const stc_didf* model, int64_t* n_cols_out, int64_t* m_out);
int stc_didf_free(stc_didf* model);

/* ---- online LDA ----------------------------------------------------------------------- */
typedef struct stc_lda_config {
  int32_t k;                     /* number of topics */
  int64_t vocab_size;            /* V (= numFeatures) */
  const double* doc_concentration; /* α: 1 value (−1 ⇒ 1/k) or k values */
  int32_t doc_concentration_len;
  double topic_concentration;    /* η (−1 ⇒ 1/k) */
  double tau0;                   /* learningOffset, default 1024 */
  double kappa;                  /* learningDecay, default 0.51 */
  double mini_batch_fraction;    /* subsamplingRate, default 0.05 */
  double gamma_shape;            /* default 100 */
  int32_t optimize_doc_concentration; /* ml.LDA default 1, mllib default 0 */
  int32_t sample_with_replacement;    /* mllib default 1 */
  uint64_t seed;                 /* λ₀ / membership / γ₀ counter-RNG seed */
  int32_t dtype;                 /* STC_F64 (default: Spark's Double E-step), STC_F32 or STC_MIXED */
  int32_t max_inner_iter;        /* E-step safety cap (upstream has none); 0 ⇒ 100000 */
  int32_t mixed_resolve_iters;   /* STC_MIXED: re-solve in fp64 the documents past this many fp32 iterations
                                    (0 ⇒ 500) */
} stc_lda_config;

/* fills the upstream defaults (ml.clustering.LDA) */
void stc_lda_config_default(stc_lda_config* cfg);

typedef struct stc_step_stats {
  int64_t batch_docs;        /* docs in the minibatch on this rank */
  int64_t nonempty_docs;     /* all ranks */
  int64_t batch_entries;     /* (doc, term) entries on this rank */
  int64_t inner_iters;       /* Σ E-step iterations on this rank */
  int32_t inner_iters_max;
  int32_t cap_hits;          /* docs stopped by max_inner_iter */
  double rho;                /* learning rate used */
} stc_step_stats;

int stc_lda_create(stc_ctx* ctx, const stc_lda_config* cfg, stc_lda** out);
int stc_lda_destroy(stc_lda* lda);
/* the documents of THIS rank; corpus_size_total = Σ over ranks (Spark's corpusSize).
 * The CSR values are read in the LDA's dtype; the handle keeps a reference to `corpus`.    */
int stc_lda_set_corpus(stc_lda* lda, const stc_dcsr* corpus, int64_t corpus_size_total);
/* λ₀ ~ Gamma(gamma_shape, 1/gamma_shape) i.i.d. from the counter RNG (seed) — identical on
 * every rank, so no broadcast is needed                                                    */
int stc_lda_init_random(stc_lda* lda, uint64_t seed);
int stc_lda_set_topics(stc_lda* lda, const double* topics, int layout);
int stc_lda_get_topics(stc_lda* lda, double* topics_out, int layout);
int stc_lda_set_alpha(stc_lda* lda, const double* alpha /* k */);
int stc_lda_get_alpha(stc_lda* lda, double* alpha_out /* k */);
int stc_lda_get_eta(stc_lda* lda, double* eta_out);
int stc_lda_get_iteration(stc_lda* lda, int64_t* iteration_out);
/* k and V of the handle (the JNI shim sizes and checks its Java arrays with them) */
int stc_lda_shape(const stc_lda* lda, int32_t* k_out, int64_t* vocab_out);

/* One submitMiniBatch over an injected membership: batch_doc_ids are row indices of this
 * rank's corpus (duplicates allowed = sampling with replacement).  gamma0 (n×k, may be NULL)
 * injects γ₀; otherwise γ₀ comes from the counter RNG keyed (seed, iteration, rank, pos).
 * stats may be NULL (then the call does not wait for the GPU).                              */
int stc_lda_step(stc_lda* lda, const int64_t* batch_doc_ids, int64_t n, const double* gamma0,
                 stc_step_stats* stats);
/* One OnlineLDAOptimizer.next(): device-side Poisson/Bernoulli membership sampling with
 * fraction mini_batch_fraction, then the same step.  Every call draws a new sample (an empty
 * GLOBAL sample returns without an iteration, as Spark's `if (batch.isEmpty()) return this`);
 * the next draw is sampled during this step, so consecutive calls do not drain the stream.  */
int stc_lda_next(stc_lda* lda, stc_step_stats* stats);
/* E-step only (no model update), for tests: gamma_out n×k; stat_out (k×V as V×k layout,
 * may be NULL) receives the summed sufficient statistics Σ_d eθ_d ⊗ (cts/φ) scattered to
 * their terms (Spark's `stat` before ⊙ expElogβ); iters_out n (may be NULL).              */
int stc_lda_estep(stc_lda* lda, const int64_t* batch_doc_ids, int64_t n, const double* gamma0,
                  double* gamma_out, double* stat_out, int32_t* iters_out);

/* LocalLDAModel.logLikelihood over `docs` (any CSR with V columns, this rank's part):
 * bound = corpusPart (Σ over all ranks) + topicsPart.  γ₀ per doc: gamma0 (rows×k) if given,
 * else counter RNG keyed (gamma_seed, doc_id_base + row).  token_count = Σ values.          */
int stc_lda_bound(stc_lda* lda, const stc_dcsr* docs, uint64_t gamma_seed, int64_t doc_id_base,
                  const double* gamma0, double* bound_out, double* corpus_part_out,
                  double* topics_part_out, double* token_count_out);
/* LocalLDAModel.topicDistribution for every row of `docs`: out rows×k (zeros for empty rows) */
int stc_lda_topic_distribution(stc_lda* lda, const stc_dcsr* docs, uint64_t gamma_seed,
                               int64_t doc_id_base, const double* gamma0, double* out);
/* LocalLDAModel.describeTopics(max_terms): idx_out k×N, weight_out k×N (N = min(max,V)) */
int stc_lda_describe(stc_lda* lda, int32_t max_terms, int32_t* idx_out, double* weight_out);

/* Average device time (ms, HIP events) of the last step's phases, for the bench:
 * [0] sample+scan, [1] E-step kernel, [2] sstats (sort + segmented SpMM), [3] all-reduce,
 * [4] M-step (λ update + expElogβ).  Requires stc_lda_enable_timing(lda, 1) beforehand.    */
int stc_lda_enable_timing(stc_lda* lda, int on);
/* cumulative since creation: [0] batch docs, [1] batch entries, [2] Σ inner E-step iterations,
 * [3] docs stopped by max_inner_iter                                                         */
int stc_lda_counters(stc_lda* lda, int64_t out[4]);
int stc_lda_phase_times(stc_lda* lda, double* ms_out /* 5 */, int64_t* steps_out);
/* E-step launches per kernel family, cumulative since creation (training and inference): what actually
 * ran, so a caller can name the kernel it timed (a team launch that timed out and was re-run on the
 * one-CU kernel counts under its family, under STC_KC_WIDE and under STC_KC_TEAM_FALLBACK) */
enum stc_kernel_count {
  STC_KC_ROWS64 = 0,        /* k_estep_rows64[_pers]: fp64, k <= 104 */
  STC_KC_ROWS64_LONG = 1,   /* k_estep_rows64_long: the pass over 7-8-row-set documents (may find none) */
  STC_KC_GRID = 2,          /* k_estep_grid[_pers] (+ its long-document pass): fp32, k <= 128 */
  STC_KC_WIDE = 3,          /* k_estep_wide: many topics, one CU per document */
  STC_KC_WIDE_MC = 4,       /* k_estep_wide_mc: many topics, the rows split over a team of CUs */
  STC_KC_WIDE_TC = 5,       /* k_estep_wide_tc: many topics, the topics split over a team */
  STC_KC_TGRID64 = 6,       /* k_estep_tgrid64: fp64, the topics split, the rows64 grid in each member */
  STC_KC_TEAM_FALLBACK = 7, /* team launches re-run on k_estep_wide after a co-residency timeout */
  STC_KC_WORKGROUP = 8,     /* k_estep: documents past the fast kernels' row capacity */
  STC_KC_MIXED_RESOLVES = 9, /* STC_MIXED: fp64 re-solve passes launched (documents past the threshold) */
  STC_KC_MIXED_DOCS = 10,   /* STC_MIXED: documents re-solved in fp64 */
  STC_KC_N = 12
};
int stc_lda_kernel_counts(stc_lda* lda, int64_t out[12]);

/* ---- one process, N devices ---------------------------------------------------------------
 * The reference trains in ONE JVM (Spark local[*], LDATraining.scala:7), so its drop-in drives every GPU
 * of the node from one handle ("single-process multi-device").  stc_group_create makes
 * one context and one LDA handle per device (distinct devices: one RCCL communicator, ncclCommInitAll;
 * the same device repeated: an in-process transport, the multi-GPU decomposition on one GPU), and every
 * group call runs the per-device call on one host thread per member.  The corpus is given once, on the
 * host, and sharded by contiguous document ranges balanced by entries (document ids stay global).  Each
 * group call = the same stc_lda_* call on every member (the collectives pair up by construction). */
typedef struct stc_group stc_group;
int stc_group_create(const int* device_ids, int n_devices, const stc_lda_config* cfg, stc_group** out);
int stc_group_destroy(stc_group* g);
int stc_group_size(const stc_group* g, int* n_out);
/* How the members' collectives travel.  Debug knob: with STC_GROUP_RCCL=1 in the environment at
 * stc_group_create, a group of distinct devices of any size (one included) builds its communicator with
 * ncclCommInitAll, runs the sharded M-step's collectives over it and drives every member from its own
 * host thread — the multi-GPU drop-in path on a one-GPU machine. */
enum stc_transport {
  STC_TRANSPORT_NONE = 0,       /* one member, no collectives */
  STC_TRANSPORT_IN_PROCESS = 1, /* one device repeated: device pointers exchanged between member threads */
  STC_TRANSPORT_RCCL = 2        /* an RCCL communicator over the members' devices (ncclCommInitAll) */
};
int stc_group_transport(const stc_group* g, int* transport_out);
/* member i's handle (counters, timing); do not call its collective entry points directly */
int stc_group_member(stc_group* g, int i, stc_lda** lda_out);
/* the training corpus (rows = documents, values in the group's dtype on device) */
int stc_group_set_corpus(stc_group* g, int64_t n_rows, int64_t n_cols, const int64_t* indptr,
                         const int32_t* indices, const double* values);
/* frees the training corpus shards (inference — describe, bound, topicDistribution — needs none;
 * next / step fail with STC_ERR_STATE until a new stc_group_set_corpus) */
int stc_group_release_corpus(stc_group* g);
int stc_group_init_random(stc_group* g, uint64_t seed);
int stc_group_set_topics(stc_group* g, const double* topics, int layout);
int stc_group_get_topics(stc_group* g, double* topics_out, int layout);
int stc_group_get_alpha(stc_group* g, double* alpha_out /* k */);
int stc_group_get_iteration(stc_group* g, int64_t* iteration_out);
/* waits until every member's queued work (the last next / step included) has finished */
int stc_group_synchronize(stc_group* g);
/* OnlineLDAOptimizer.next() over every member's documents; stats summed over the members */
int stc_group_next(stc_group* g, stc_step_stats* stats);
/* submitMiniBatch over injected GLOBAL document ids (gamma0 n×k in the same order, may be NULL) */
int stc_group_step(stc_group* g, const int64_t* batch_doc_ids, int64_t n, const double* gamma0,
                   stc_step_stats* stats);
int stc_group_describe(stc_group* g, int32_t max_terms, int32_t* idx_out, double* weight_out);
/* logLikelihood / topicDistribution of host documents, sharded over the members; γ₀ keys are
 * doc_id_base + global row, so the results equal a single handle's over the same rows */
int stc_group_bound(stc_group* g, int64_t n_rows, int64_t n_cols, const int64_t* indptr,
                    const int32_t* indices, const double* values, uint64_t gamma_seed, int64_t doc_id_base,
                    const double* gamma0, double* bound_out, double* corpus_part_out,
                    double* topics_part_out, double* token_count_out);
int stc_group_topic_distribution(stc_group* g, int64_t n_rows, int64_t n_cols, const int64_t* indptr,
                                 const int32_t* indices, const double* values, uint64_t gamma_seed,
                                 int64_t doc_id_base, const double* gamma0, double* out /* rows×k */);

#ifdef __cplusplus
}
#endif
#endif /* STC_H_ */
