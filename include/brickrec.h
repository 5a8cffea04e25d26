/*
 * brickrec.h — C-ABI of libbrickrec.so, the MI355X (gfx950) scoring engine behind the
 * similar-sets / hybrid-recommendation hot path of davidry777/Brickbrain-Rec-Engine.
 *
 * The reference has no FFI: its boundary is the Python class interface in
 * src/scripts/recommendation_system.py and the FastAPI routes in
 * src/scripts/recommendation_api.py.  The Python drop-ins in
 * brickbrain-rec-engine_amd/brickrec/ keep those signatures and call this ABI through
 * ctypes.  Each entry point below names the reference code it
 * replaces.
 *
 * Conventions
 *   - every function returns int status: 0 = ok, < 0 = error (BB_E_*); no C++ exception
 *     crosses the ABI; bb_last_error() returns a thread-local message for the last error.
 *   - the library owns the device copies it makes; the caller owns every pointer it
 *     passes (host or device, as the `where` field says) and keeps it alive for the call.
 *   - a handle is NOT re-entrant: one call at a time per handle (the Python side holds a
 *     lock, matching the reference's single-connection, event-loop-serialised engine,
 *     recommendation_api.py:44-67).  A handle owns one HIP stream on its device.
 *   - item ids are 0-based row indices of the uploaded item matrix plus the handle's
 *     id_offset (row sharding across GPUs).  Empty result slots hold id -1, score 0.
 *   - ordering is (score desc, id asc) everywhere (SURVEY.md §8a rule v).
 */
#ifndef BRICKREC_H
#define BRICKREC_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define BB_ABI_VERSION 2

/* status codes */
#define BB_OK 0
#define BB_E_ARG (-1)      /* invalid argument / shape */
#define BB_E_HIP (-2)      /* HIP runtime error (message in bb_last_error) */
#define BB_E_STATE (-3)    /* call out of order (e.g. search before upload) */
#define BB_E_NOMEM (-4)    /* device allocation failed */
#define BB_E_HOSTSYNC (-5) /* bb_plan_create: the search synchronises with the host mid-way (no plan: use bb_search) */

/* element types */
#define BB_F32 0
#define BB_BF16 1
#define BB_F64 2           /* host input only: converted (after f64 normalisation) */

/* pointer location */
#define BB_HOST 0
#define BB_DEVICE 1

/* search modes */
#define BB_MODE_SEMANTIC 0 /* cosine KNN of query rows (pgvector/FAISS path,
                              lego_nlp_recommeder.py:1379-1412)                       */
#define BB_MODE_SIMILAR 1  /* similar sets of item ids: cosine, drop rank 0, mask
                              (ContentBasedRecommender.get_similar_sets,
                               recommendation_system.py:194-249)                      */
#define BB_MODE_CF 2       /* u·F, exclude rated, mask, stable desc
                              (CollaborativeFilteringRecommender.get_recommendations,
                               recommendation_system.py:411-483)                      */
#define BB_MODE_HYBRID 3   /* similar(2k) ∪ cf(2k) union-blend wc·c + wcf·cf
                              (HybridRecommender.get_recommendations +
                               _combine_recommendations, :612-677, :789-843)          */

/* bb_query.flags */
#define BB_Q_OUT_KEYS 1    /* write per-side candidate key lists (for a cross-GPU
                              merge with bb_finalize) instead of final results       */
#define BB_Q_NULL_STREAM 2 /* run on the device's null stream (stream field ignored) */

typedef struct bb_index bb_index;

typedef struct {
  int32_t device;          /* HIP device ordinal; -1 = current device                 */
  int32_t dtype;           /* item storage + MFMA input type: BB_F32 or BB_BF16        */
  int64_t id_offset;       /* global id of local row 0 (row-sharded index)             */
  int64_t workspace_bytes; /* cap for the score-slab workspace; 0 = 512 MiB             */
} bb_desc;

/* Item matrix.  Replaces ContentBasedRecommender._create_feature_matrix's feat_matrix
 * (recommendation_system.py:175-192) and the PGVector embedding collection
 * (lego_nlp_recommeder.py:288-305).  rows: n×d row-major (host or device per `where`),
 * in_dtype BB_F32/BB_F64/BB_BF16.  Rows are L2-normalised once here (in f64 for f64
 * input) exactly as cosine_similarity normalises them on every call (:214), unless
 * prenormalized != 0.  Zero rows stay zero (score 0), as in sklearn.
 * present_bits (host, ⌈n/32⌉ words, NULL = all): rows that exist in the content item space
 * (feat_matrix rows, WHERE num_parts > 0 at :115); other rows (e.g. sets that only the CF
 * pivot knows) are never returned by the content side and never count as its rank 0.
 * Device-resident rows (where = BB_DEVICE) are read on the index's own stream: the caller
 * makes them complete first (e.g. synchronises the stream that produced them). */
int bb_create(const bb_desc* desc, bb_index** out);
int bb_upload_items(bb_index* idx, const void* rows, int64_t n, int32_t d, int32_t in_dtype,
                    int32_t prenormalized, int32_t where, const uint32_t* present_bits);

/* CF item factors, n×r in the SAME item row space as bb_upload_items (the drop-in
 * scatters TruncatedSVD components_.T rows, recommendation_system.py:399-407, into it).
 * present_bits: ⌈n/32⌉ words, bit i = item i exists in the CF item space (pivot columns,
 * :325-336); NULL = all present.  Host pointers. */
int bb_upload_cf(bb_index* idx, const void* item_factors, int32_t r, int32_t in_dtype,
                 const uint32_t* present_bits);

/* Item attribute columns read by the hard-constraint predicates
 * (hard_constraint_filter.py:366-480 via the sets table, rebrickable_schema.sql:38-46).
 * theme_id < 0 means SQL NULL.  Host pointers, n entries each. */
int bb_upload_attrs(bb_index* idx, const int32_t* num_parts, const int16_t* year,
                    const int32_t* theme_id);

/* Hard-constraint predicate spec: the on-device form of _build_constraint_sql /
 * _constraint_to_sql (hard_constraint_filter.py:318-480).  All bounds inclusive; the
 * always-on "num_parts > 0" (:343) is implied.  theme_bits: bitmap over theme ids
 * [0, n_theme_bits); theme_mode 0 = no theme test, 1 = require theme in set (no match
 * or NULL theme -> false, :402-409), 2 = exclude theme in set (NULL theme -> false,
 * SQL three-valued NOT, :411-418).  excluded_items: global ids cleared afterwards
 * (user_collections / user_wishlists NOT EXISTS, :441-451). */
typedef struct {
  int32_t parts_min, parts_max;   /* use INT32_MIN / INT32_MAX for "none" */
  int32_t year_min, year_max;
  int32_t theme_mode;
  int32_t n_theme_bits;
  const uint32_t* theme_bits;     /* host */
  const int64_t* excluded_items;  /* host, global ids */
  int64_t n_excluded;
} bb_predicate;

/* Evaluate predicates into a mask bitset (⌈n/32⌉ words, bit=1 -> item allowed) at
 * out_bits (device pointer if where == BB_DEVICE, else host).  Replaces the SQL round
 * trip of HardConstraintFilter.apply_constraints (hard_constraint_filter.py:263-316)
 * and the O(N·|valid|) list membership tests (recommendation_system.py:229, 454). */
int bb_eval_mask(bb_index* idx, const bb_predicate* pred, uint32_t* out_bits, int32_t where);

typedef struct {
  int32_t mode;          /* BB_MODE_* */
  int32_t flags;         /* BB_Q_* */
  int32_t B;             /* number of queries */
  int32_t k;             /* final list length (reference top_k; API caps it at 50) */
  int32_t k_side;        /* hybrid per-side list length; 0 = 2k (:648-656)            */
  int32_t where;         /* location of every pointer below (BB_HOST / BB_DEVICE)     */
  const void* q_rows;    /* SEMANTIC: B×d query rows, q_dtype (normalised in-kernel)  */
  int32_t q_dtype;
  const int64_t* q_items;   /* SIMILAR / HYBRID: B global item ids (liked set)        */
  const void* q_cf;      /* CF / HYBRID: B×r user factor rows (user_factors[user_idx],
                            :432-438), q_cf_dtype                                    */
  int32_t q_cf_dtype;
  const uint32_t* mask_bits;   /* ⌈n/32⌉ words, NULL = no filter (:229, :454)          */
  const uint32_t* excl_bits;   /* B×⌈n/32⌉ words: per-query excluded items (CF: items
                                  the user rated, :441-451); NULL = none              */
  double w_content, w_cf;      /* hybrid weights (0.4 / 0.6 at :609-610)               */
  void* stream;          /* hipStream_t to run on; NULL = the handle's stream          */
  int64_t mask_count;    /* ABI 2: allowed items in mask_bits when the caller knows it (the
                            length of the reference's valid_set_nums, :634), 0 = unknown.
                            Host masks are counted by the library.  With a count the search
                            may score only the allowed rows (BB_OPT_PREFILTER); a device
                            mask_count must be >= the true count (if the device finds more
                            allowed items than it, every result row comes back empty)      */
} bb_query;

typedef struct {
  float* scores;         /* B×k (final) */
  int64_t* ids;          /* B×k (final), -1 = empty slot */
  int32_t* counts;       /* B, number of filled slots; may be NULL */
  int32_t where;         /* location of the three pointers above */
  /* BB_Q_OUT_KEYS only: device buffers the caller sizes with bb_key_lens() */
  uint64_t* keys;        /* [sides][B][k_int] ordered keys (0 = empty)                 */
  uint64_t* max_keys;    /* [B] unmasked arg-max key per query (rank-0 drop)           */
} bb_result;

/* Batched scoring + top-k.  Replaces the cosine_similarity + argsort + Python filter
 * loop of get_similar_sets (:213-247), the np.dot + loop + sort of the CF
 * get_recommendations (:438-461), the union-blend (:789-843) and the PGVector
 * retriever KNN (lego_nlp_recommeder.py:1394).  Asynchronous on the stream when every
 * pointer is a device pointer; synchronises before returning when results are host. */
int bb_search(bb_index* idx, const bb_query* q, bb_result* res);

/* Lengths of the BB_Q_OUT_KEYS lists for a query: sides (1 or 2) and k_int per side. */
int bb_key_lens(const bb_query* q, int32_t* sides, int32_t* k_int);

/* Cross-shard merge: keys gathered from P shards ([P][sides][B][k_int]) and their
 * max_keys ([P][B]) -> final results, applying the same rank-0 drop, truncation and
 * hybrid blend bb_search applies locally.  keys / max_keys live where
 * q->where says (host lists are staged to the device); results where res->where says.
 * BB_Q_OUT_KEYS searches write their lists to host buffers too when res->where is
 * BB_HOST (synchronised before returning). */
int bb_finalize(bb_index* idx, const bb_query* q, const uint64_t* keys, const uint64_t* max_keys,
                int32_t n_parts, bb_result* res);

/* Profiling: when enabled, per-kernel HIP events are recorded on the launch stream;
 * bb_get_profile synchronises and returns the accumulated device time and launch count
 * of each kernel family, then clears them. names: "prep","gemm","select","finalize","mask","rerun","rerank","pack" (the constraint-first packing launch). */
typedef struct {
  double ms[8];
  int64_t launches[8];
  const char* names[8];
  int32_t n;
} bb_profile;
int bb_set_profiling(bb_index* idx, int32_t on);
int bb_get_profile(bb_index* idx, bb_profile* out);

/* Search-path options (no reference counterpart: tuning knobs of this implementation).
 *   BB_OPT_STREAM           -1 auto (default), 0 never, 1 always: the streaming top-K for
 *                           large indexes (pilot bound + candidate regions, no B×n score
 *                           slab); auto = when the index has >= BB_OPT_STREAM_MIN_ITEMS rows.
 *                           Results are identical either way.
 *   BB_OPT_STREAM_MIN_ITEMS rows from which auto streams (default 100000)
 *   BB_OPT_WORKSPACE_BYTES  score-slab workspace cap (default 512 MiB; streaming may use up
 *                           to 4 GiB unless this is set)
 *   BB_OPT_STREAM_REFINE    -1 auto (default), 0 never, 1 always (index >= 2x the pilot): the
 *                           two-level streaming bound.  Results are identical either way.
 *   BB_OPT_RR_LISTS         -1 auto (default, = 1), 0 off: one-slab searches of an f32 index
 *                           keep bounded per-lane candidate lists in the scan instead of
 *                           writing a score image for the select (no B×n image).  Results are
 *                           identical either way.
 *   BB_OPT_SMALL_BATCH      -1 auto (default, = 1), 0 off: batches of up to 16 query rows (any
 *                           mode, hybrid included) on an f32 index of up to 65,536 rows take
 *                           one approximate pass over the f16 copy per side and an exact
 *                           rescore of the candidates within its proven bound (no MFMA scan,
 *                           lists or list select) — the reference's one-query request shape.
 *                           Results are identical either way.
 *   BB_OPT_PREFILTER        -1 auto (default), 0 off, 1 whenever the mask's count is known:
 *                           constraint-first search (the reference's step 1, "apply hard
 *                           constraints first", recommendation_system.py:628-656).  The rows
 *                           the mask allows are packed in one launch and only they are
 *                           scanned, listed and rescored; auto = when at most n/4 rows are
 *                           allowed, on f32 indexes of up to 65,536 rows, batches of more
 *                           than 16 rows.  Similar / hybrid queries drop their rank-0 item
 *                           (the unmasked arg-max) from a per-item table built at upload.
 *                           Results are identical either way. */
#define BB_OPT_STREAM 1
#define BB_OPT_STREAM_MIN_ITEMS 2
#define BB_OPT_WORKSPACE_BYTES 3
#define BB_OPT_STREAM_REFINE 4
#define BB_OPT_RR_LISTS 5
#define BB_OPT_SMALL_BATCH 6
#define BB_OPT_PREFILTER 7
int bb_set_option(bb_index* idx, int32_t option, int64_t value);

/* Stored (normalised, index-dtype) item rows of B global ids into out (B×d, row-major;
 * ids outside this index's rows give zero rows).  ids and out live at `where`.  Lets a
 * row-sharded deployment hand the owning shard's row of a liked set to every shard
 * (SIMILAR / HYBRID queries with q_rows instead of q_items), the sharded analogue of
 * feat_matrix[target_idx] (recommendation_system.py:213).  Synchronous; device ids are
 * read on the index's own stream, so they must be complete when the call is made. */
int bb_get_rows(bb_index* idx, const int64_t* ids, int32_t B, void* out, int32_t where);

/* A second handle over the same resident rows (no reference counterpart: serving plumbing).
 * The view has its own HIP stream and scratch workspace but aliases the base's item rows, CF
 * factors, attribute columns and bitsets, so several batches can be in flight on one device
 * with ONE copy of the index in HBM / the MALL instead of one per in-flight handle.  Uploads to
 * a view, or to a base while it has views, fail with BB_E_STATE; destroy the views first. */
int bb_create_view(bb_index* base, bb_index** out);

/* Prepared searches (no reference counterpart: the serving loop's repeated request).  The
 * reference answers one request per call — get_similar_sets of one target row
 * (recommendation_system.py:213-217), the retriever's one embedding (lego_nlp_recommeder.py:305)
 * — and so does a server here: the same query shape with new contents every time.
 * bb_plan_create runs the host side of bb_search once (path choice, sizes, kernel arguments)
 * and records its launches instead of issuing them; bb_plan_launch replays them, reading the
 * query buffers' CURRENT contents and writing the results, at the cost of the launches alone.
 * q and res must name device buffers (where = BB_DEVICE) that stay allocated while the plan
 * lives; the plan runs on q->stream (NULL: its own stream; BB_Q_NULL_STREAM: the null stream).
 * The plan owns a private view of the index (its own workspace): plans never race with
 * bb_search or with each other on scratch buffers, and the index accepts no upload while a
 * plan exists (BB_E_STATE, as with views).  Searches that synchronise with the host (the
 * streaming top-K of indexes >= BB_OPT_STREAM_MIN_ITEMS rows) return BB_E_HOSTSYNC: use
 * bb_search for those; any other refusal is an error.  One plan may be launched from several
 * threads: bb_plan_launch holds the plan's lock while it enqueues, so two replays never
 * interleave their launches on the plan's workspace (they still share it: the second replay
 * queues behind the first on the stream).  The plan's stream must stay valid until
 * bb_plan_destroy, which waits for that stream (not for the whole device), then releases the
 * view. */
typedef struct bb_plan bb_plan;
int bb_plan_create(bb_index* idx, const bb_query* q, const bb_result* res, bb_plan** out);
int bb_plan_launch(bb_plan* plan);
int bb_plan_destroy(bb_plan* plan);

/* Diagnostics (no device call): BB_OK when the hybrid dual list scan accepts a configs[2]-shaped
 * argument pair (1,024 query rows, 25,216 items, f16 content rows 384 wide, CF 64) with item row
 * stride `ldx`, else BB_E_ARG naming the broken rule — the scan's LDS-DMA source offsets are 24-bit,
 * so a stride >= 2^23 is refused before any launch instead of faulting. */
int bb_check_dual_scan_args(int64_t ldx);

int bb_info(bb_index* idx, int64_t* n_items, int32_t* d, int32_t* d_pad, int32_t* r);
/* Handles are checked by every entry point: a destroyed, foreign or corrupted bb_index /
 * bb_plan pointer returns BB_E_ARG with a message in bb_last_error(), never a crash.  A handle
 * is invalid from the moment its destroy call begins (removal from the live set is the point
 * of truth: of two concurrent destroys of one handle, one succeeds and the other returns
 * BB_E_ARG), even if its address is later reused by a new handle; calling other entry points
 * on a handle while another thread destroys it is misuse. */
int bb_destroy(bb_index* idx);
const char* bb_last_error(void);
int bb_abi_version(void);

#ifdef __cplusplus
}
#endif
#endif /* BRICKREC_H */
