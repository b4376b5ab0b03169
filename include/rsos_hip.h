/*
 * rsos_hip.h -- C ABI of librsos_hip.so, the MI355X (gfx950) fingerprint-hash path of
 * reconcile-rs.
 *
 * What it replaces (citations relative to the reference checkout, Akvize/reconcile-rs 0.3.0):
 *   - rsos::lift / rsos::digest                      rsos/src/fingerprint.rs:270-292
 *     (BLAKE3 over the canonical encoding, rsos/src/encoding.rs:17-35)
 *   - Fingerprint + / - (mod 2^256, LE u64 limbs)    rsos/src/fingerprint.rs:145-173
 *   - Aggregate (fingerprint, size) monoid           rsos/src/aggregate.rs:38-89
 *   - FingerprintTreeMap's cached subtree aggregates rsos/src/fingerprint_tree_map/node.rs:54-91
 *     and its range query                            rsos/src/fingerprint_tree_map/query.rs:25-76
 *   - the Rsos<K> trait surface (size / aggregate / rank / select / insert / delete)
 *                                                    rsos/src/rsos_trait.rs:39-90
 *     which rbsr consumes through RsosView<K>        rbsr/src/rsos_view.rs:55-91
 *   - rbsr's protocol round, its questions batched   rbsr/src/protocol.rs:212-317
 *   - the snapshot reload and the RangeAggregate wire codec
 *                                                    src/snapshot.rs:30-98, gossip/src/bincode.rs:65-100
 *
 * Conventions
 *   - Every call returns rh_status (0 = ok, negative = error); rh_last_error() gives a
 *     thread-local message.  No exceptions, no callbacks cross this boundary.
 *   - A fingerprint is 32 bytes: the BLAKE3 digest read as four little-endian u64 limbs,
 *     limb 0 least significant (rsos/src/fingerprint.rs:106-124).  On the wire and in these
 *     buffers the 32 bytes are exactly the digest bytes.
 *   - rh_aggregate mirrors rsos::Aggregate's field order (fingerprint, then size;
 *     rsos/src/aggregate.rs:38-42).
 *   - *_async calls take DEVICE pointers and enqueue on `stream` (a hipStream_t, or NULL for
 *     the null stream); they never synchronise, allocate or copy to the host.
 *   - rh_store_* calls take HOST pointers and are synchronous: the stream is drained before
 *     return, so a caller holding the map's read lock never observes an in-flight batch
 *     (the one-snapshot-per-round law, rbsr/src/rsos_view.rs:36).
 */
#ifndef RSOS_HIP_H
#define RSOS_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define RH_ABI_VERSION 1

typedef enum rh_status {
    RH_OK = 0,
    RH_ERR_ARG = -1,         /* bad argument (null pointer, misaligned buffer, bad range)     */
    RH_ERR_HIP = -2,         /* a HIP runtime call failed (message in rh_last_error)           */
    RH_ERR_OOM = -3,         /* device (or page-locked host) allocation failed                 */
    RH_ERR_UNSUPPORTED = -4, /* schema has no specialised kernel: encode on the host and use
                                rh_lift_encoded_async (the generic canonical-bytes path)       */
    RH_ERR_STATE = -5,       /* call not valid in the store's current state                   */
    RH_ERR_DATA = -6         /* malformed snapshot / wire bytes (the reference's
                                io::ErrorKind::InvalidData / bincode error)                    */
} rh_status;

/* Key encodings (rsos/src/encoding/serializer.rs):
 *   UNIT  : `()`            -> no bytes (digest = lift with a unit key, fingerprint.rs:288-292)
 *   U32   : u32 / i32       -> 4 bytes LE              (:76-79)
 *   U64   : u64 / i64/usize -> 8 bytes LE              (:81-84)
 *   BYTES : [u8; L] / Vec<u8> / String of fixed byte length L
 *                           -> u64 LE length L, then the L bytes (:105-113,162-179)        */
typedef enum rh_key_kind { RH_KEY_UNIT = 0, RH_KEY_U32 = 1, RH_KEY_U64 = 2, RH_KEY_BYTES = 3 } rh_key_kind;
typedef enum rh_value_kind { RH_VAL_UNIT = 0, RH_VAL_U32 = 1, RH_VAL_U64 = 2, RH_VAL_BYTES = 3 } rh_value_kind;

/* What is hashed per record:
 *   PLAIN      : lift(k, v)                                   FingerprintTreeMap<K, V>
 *   DATED      : lift(k, Entry<Timestamp, V>{stamp, state})   Replica.map   (src/replica.rs:69)
 *   PROJECTION : lift(k, State<V>)                            Replica.projection (:74)
 * Entry/State/Timestamp: lww-register/src/entry.rs:24-29,88-94; clock.rs:143-181.        */
typedef enum rh_record_kind { RH_REC_PLAIN = 0, RH_REC_DATED = 1, RH_REC_PROJECTION = 2 } rh_record_kind;

typedef struct rh_schema {
    int32_t  key_kind;    /* rh_key_kind                                  */
    uint32_t key_len;     /* bytes per key in the key column (4, 8 or L)  */
    int32_t  value_kind;  /* rh_value_kind                                */
    uint32_t value_len;   /* bytes per value in the value column          */
    int32_t  record_kind; /* rh_record_kind                               */
    uint32_t reserved;    /* must be 0                                    */
} rh_schema;

/* Records in column (SoA) layout, row i = record i.  Columns a schema does not use may be NULL.
 * Device columns must be 16-byte aligned (hipMalloc / torch allocations are).             */
typedef struct rh_columns {
    const void     *keys;    /* n * key_len bytes                                        */
    const uint64_t *phys;    /* DATED: Timestamp.hlc.physical (PhysicalTime, ms)         */
    const uint32_t *logical; /* DATED: Timestamp.hlc.logical  (LogicalCounter)           */
    const uint64_t *node;    /* DATED: Timestamp.node_id      (NodeId)                   */
    const uint8_t  *tags;    /* DATED/PROJECTION, nullable: 0 = State::Present, 1 = Tombstone */
    const void     *values;  /* n * value_len bytes                                      */
} rh_columns;

typedef struct rh_aggregate {
    uint64_t fingerprint[4]; /* Aggregate.fingerprint, LE limbs */
    uint64_t size;           /* Aggregate.size                  */
} rh_aggregate;

/* ---- library ------------------------------------------------------------------------- */
int         rh_abi_version(void);
const char *rh_last_error(void);
/* 1 if a specialised kernel exists for this schema, 0 if it needs the encoded path, <0 bad */
int         rh_schema_supported(const rh_schema *schema);
/* canonical-encoding length of a present / tombstone record of this schema (host helper)   */
int64_t     rh_schema_record_len(const rh_schema *schema, int tombstone);

/* ---- device-resident batch API (all pointers are device pointers) -------------------- */
/* Records are grouped in blocks of RH_BLOCK = 256 consecutive rows, blocks in
 * super-blocks of 256 blocks (65536 rows); these are the cached "subtree" aggregates. */
#define RH_BLOCK 256
#define RH_SUPER 65536
size_t rh_num_blocks(size_t n);      /* ceil(n / 256)   */
size_t rh_num_superblocks(size_t n); /* ceil(n / 65536) */

/* lift every record: fps[i] = lift(key_i, record_i)  (32 B each, rsos/src/fingerprint.rs:270);
 * block_sums (nullable) receives Σ fps over each 256-row block (32 B per block).
 * Replaces the per-insert lift of FingerprintTreeMap::insert (mutate.rs:34,61) and
 * Replica::map_insert's two lifts (src/replica/write.rs:44-45).                           */
int rh_lift_records_async(const rh_schema *schema, const rh_columns *dev_cols, size_t n,
                          uint8_t *dev_fps, uint8_t *dev_block_sums, void *stream);

/* Both lifts of Replica::map_insert in one pass (src/replica/write.rs:44-45): the dated
 * fingerprint lift(k, Entry<Timestamp,V>) and the projection lift(k, State<V>).
 * schema->record_kind must be RH_REC_DATED.  Either block-sum pointer may be NULL.        */
int rh_lift_dual_async(const rh_schema *schema, const rh_columns *dev_cols, size_t n,
                       uint8_t *dev_fps_dated, uint8_t *dev_block_sums_dated,
                       uint8_t *dev_fps_proj, uint8_t *dev_block_sums_proj, void *stream);

/* Generic path: BLAKE3 of pre-encoded canonical bytes (rsos::encoding::encode_to_vec of
 * k then v, public-api/rsos.txt:61), record i = bytes[offsets[i] .. offsets[i+1]).
 * dev_bytes 4-byte aligned; bytes_len: its readable size, a multiple of 4 and >= offsets[n]
 * (pad the buffer).  Nothing is read at or past bytes_len: offsets that decrease or exceed it are a
 * caller error that yields wrong fingerprints, not a fault.  Fully asynchronous.          */
int rh_lift_encoded_async(const uint8_t *dev_bytes, size_t bytes_len, const uint64_t *dev_offsets, size_t n,
                          uint8_t *dev_fps, uint8_t *dev_block_sums, void *stream);

/* Generic path for fixed-length encodings (a K / V pair whose canonical encoding always has
 * one length: fixed-width integers, arrays, fixed-size structs): record i =
 * bytes[i * record_len .. (i + 1) * record_len), no offsets.  dev_bytes 4-byte aligned;
 * bytes_len: its readable size, a multiple of 4 and >= n * record_len (RH_ERR_ARG otherwise).               */
int rh_lift_fixed_async(const uint8_t *dev_bytes, size_t bytes_len, size_t record_len, size_t n,
                        uint8_t *dev_fps, uint8_t *dev_block_sums, void *stream);

/* out[g] = Σ in[256 g .. 256 g + 255]  (32-byte fingerprints, mod 2^256) */
int rh_reduce_blocks_async(const uint8_t *dev_in, size_t n_in, uint8_t *dev_out, void *stream);

/* Range aggregates over rank ranges [lo[j], hi[j]) of a lifted, rank-ordered array:
 * out[j] = (Σ fps[lo..hi), hi - lo).  Uses the block and super-block sums, so the cost per
 * range is O(n / 65536 + 512) reads -- the cached-subtree walk of query.rs:25-76.
 * An inverted or empty range yields the zero aggregate (rbsr/src/protocol.rs:230-232).   */
int rh_range_aggregates_async(const uint8_t *dev_fps, const uint8_t *dev_block_sums,
                              const uint8_t *dev_super_sums, size_t n, const uint64_t *dev_lo,
                              const uint64_t *dev_hi, size_t r, rh_aggregate *dev_out, void *stream);

/* out[j] = Σ_p in[p * r + j]  (the combine step after a cross-GPU gather of per-shard
 * aggregates; Aggregate's Add, rsos/src/aggregate.rs:79-89)                               */
int rh_combine_aggregates_async(const rh_aggregate *dev_in, size_t parts, size_t r,
                                rh_aggregate *dev_out, void *stream);

/* ---- host helpers --------------------------------------------------------------------- */
/* End-to-end lift of host records: H2D copy, lift on `device`, D2H of the fingerprints,
 * pipelined in ~128 MB chunks over three streams (copy in / lift / copy out, so PCIe carries
 * both directions at once).  The PCIe-inclusive path a host caller (the Rust shim) uses for a
 * one-shot batch; host buffers from rh_host_alloc (pinned) let the copies overlap.         */
int rh_lift_host(int device, const rh_schema *schema, const rh_columns *host_cols, size_t n,
                 uint8_t *host_fps);

/* Page-locked host memory for rh_lift_host / rh_store_load / rh_store_apply buffers.     */
int rh_host_alloc(size_t bytes, void **out);
int rh_host_free(void *p);

/* Fingerprint group on the host (rsos/src/fingerprint.rs:145-173), for callers' combines */
void rh_fp_add(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]);
void rh_fp_sub(const uint64_t a[4], const uint64_t b[4], uint64_t out[4]);

/* ---- GPU-resident RSOS store ---------------------------------------------------------
 * A rank-ordered set resident in HBM: keys, per-record fingerprints, and the 256-row block /
 * 65536-row super-block sums (the GPU form of FingerprintTreeMap's cached subtree
 * Aggregates, rsos/src/fingerprint_tree_map/node.rs:54-91).  Record payloads are lifted on
 * ingest and not kept on the device; the caller owns K and V in host memory, as the
 * reference's map does (Rsos::enumerate / select return borrows, rsos_trait.rs:66-80).
 * Realises Rsos<K> (rsos/src/rsos_trait.rs:39-90) for u32 / u64 / 8-, 16-, 32-byte keys:
 *   size -> rh_store_len, aggregate -> rh_store_aggregate[s|_keys], rank -> rh_store_rank[s],
 *   select -> rh_store_select, insert / delete -> rh_store_apply[_device].
 * Every call drains the store's stream before returning.
 * Device memory: keys + 32 B fingerprint per base row, block sums, search samples and tables,
 * the delta run (a 40 B record per changed key), and -- for questions over the device -- a row
 * prefix of the base, 32 B per row (3.2 GB at 10^8 rows), allocated at a base's first device
 * question only while 1 GiB stays free (RSOS_HIP_ROW_PREFIX=0: none; sums then take a block prefix
 * and the head / tail rows).  Streams: the store's own at the device's highest priority;
 * background kernels (the host tier's refresh scans, the row prefix) on streams whose CU mask
 * leaves the last RSOS_HIP_BG_RESERVE (default 32) compute units to the questions' kernels.     */
typedef struct rh_store rh_store;
/* Row cap: one rh_store holds fewer than 2^31 rows (RH_STORE_MAX_ROWS; its device ranks and counts
 * are 32-bit).  rh_store_load / _load_device / _reserve with n >= 2^31, and rh_store_apply /
 * _apply_device / a staged batch that would take the store to 2^31 rows, return RH_ERR_ARG
 * ("store size limit (2^31 rows) exceeded ...") and change nothing.  Rsos::size() is a usize
 * (rsos/src/rsos_trait.rs:44): a map of 2^31 rows or more (one MI355X holds ~2.1 x 10^9 rows of
 * 16 B keys) is an rh_sstore (below; HipShardedMap in Rust), each shard under the cap.        */
#define RH_STORE_MAX_ROWS 2147483648 /* 2^31 */

int rh_store_create(int device, const rh_schema *schema, rh_store **out);
int rh_store_destroy(rh_store *store);
/* Replace the contents with n records, sorted by key in the key type's Ord and free of
 * duplicates (checked on the device; RH_ERR_ARG otherwise).  Bulk fill: the GPU form of
 * FromIterator / ReplicatedMap::load_bulk (rsos/src/fingerprint_tree_map_iter/into_iter.rs:22-33,
 * src/replicated_map/write.rs:184).  _device: the columns are already in HBM.             */
int rh_store_load(rh_store *store, const rh_columns *host_cols, size_t n);
/* dev_cols were written on `after_stream` (a hipStream_t; NULL = the null stream): the store's
 * own stream waits for the work already queued there before reading them.                 */
int rh_store_load_device(rh_store *store, const rh_columns *dev_cols, size_t n, void *after_stream);
int rh_store_len(rh_store *store, uint64_t *out);
/* Aggregate over rank range [lo, hi) */
int rh_store_aggregate(rh_store *store, uint64_t lo, uint64_t hi, rh_aggregate *out);
/* r rank ranges in one launch (the <= 16 child ranges of one rbsr SPLIT, protocol.rs:299-307) */
int rh_store_aggregates(rh_store *store, const uint64_t *lo, const uint64_t *hi, size_t r,
                        rh_aggregate *out);
/* Aggregate over the key range given by two bounds.  kind: 0 = unbounded, 1 = included,
 * 2 = excluded (std::ops::Bound).  Inverted ranges give ZERO (rbsr/src/protocol.rs:230-232). */
int rh_store_aggregate_keys(rh_store *store, int lo_kind, const void *lo_key, int hi_kind,
                            const void *hi_key, rh_aggregate *out);
/* Rank(z) = number of keys strictly below z (query.rs:93-121); _ranks: m keys at once      */
int rh_store_rank(rh_store *store, const void *key, uint64_t *out);
int rh_store_ranks(rh_store *store, const void *keys, size_t m, uint64_t *out);
/* Select(r): copies the r-th key into key_out (key_len bytes); RH_ERR_ARG if r >= size      */
int rh_store_select(rh_store *store, uint64_t r, void *key_out);
/* Copy the keys / fingerprints of ranks [lo, hi) to the host (Enumerate's key order)       */
int rh_store_keys(rh_store *store, uint64_t lo, uint64_t hi, void *host_out);
int rh_store_fingerprints(rh_store *store, uint64_t lo, uint64_t hi, uint8_t *host_out);

/* ---- rbsr protocol round, batched ---------------------------------------------------------
 * protocol_round_with_policy (rbsr/src/protocol.rs:212-317) asks its RsosView, for every active
 * segment, aggregate(start..end) and the ranks of both bounds (BoundedRange::parse,
 * rbsr/src/protocol/rank.rs), and for every SPLIT child select(cut) and aggregate(child).  These
 * two calls answer one round's questions in two device round trips, against one state of the
 * store (the one-snapshot-per-round law, rsos_view.rs:36); the policy (any RefinementPolicy)
 * and the round's bookkeeping stay with the host driver.
 * resolve: r segments in the wire codec's form -- start kind 0 = Unbounded, 1 = Included(key);
 * end kind 0 = Unbounded, 1 = Excluded(key); keys r * key_len bytes (rows of unbounded sides
 * are ignored).  Out: raw_start = Unbounded ? 0 : rank(start), raw_end = Unbounded ? size :
 * rank(end), and the local aggregate over the key range (ZERO for an inverted segment,
 * raw_end < raw_start, which the driver drops).
 * split: m select() ranks (each < size, RH_ERR_ARG otherwise) -> m keys (m * key_len bytes),
 * and q rank ranges [lo, hi) -> q aggregates.                                                */
int rh_store_resolve_segments(rh_store *store, size_t r, const uint8_t *start_kinds, const void *start_keys,
                              const uint8_t *end_kinds, const void *end_keys, uint64_t *raw_start,
                              uint64_t *raw_end, rh_aggregate *local);
int rh_store_split_segments(rh_store *store, size_t m, const uint64_t *select_ranks, void *keys_out, size_t q,
                            const uint64_t *lo, const uint64_t *hi, rh_aggregate *out);

/* A whole round in one call and one device round trip (decisions, cut keys and children formed on
 * the device), for the shipped policies that decide on the span alone:
 * FixedFanOut(fan_out) (rbsr/src/policy/fixed_fan_out.rs; fan_out < 2 is raised to 2, 16 =
 * FanOut::NEGENTROPY, the default of protocol_round) and SqrtFanOut (sqrt_fan_out.rs).  Segments
 * travel in the wire codec's SoA form (rh_wire_*): `active` in (n items); children (SPLIT
 * children and bounced IDLIST parents, with aggregates) and enumeration ranges (IDLIST;
 * aggregates NULL) out, in the reference's order.  The output arrays belong to the store: the
 * call fills both rh_segments with pointers to them (cap = n = the item count), valid until the
 * next call on this store -- so a round's children may be passed straight to the peer store's
 * round, never back to the store that produced them.                                         */
typedef enum rh_policy { RH_POLICY_FIXED_FAN_OUT = 0, RH_POLICY_SQRT_FAN_OUT = 1 } rh_policy;
typedef struct rh_segments {
    uint8_t *start_kinds;     /* 0 = Unbounded, 1 = Included(key)                        */
    void *start_keys;         /* cap * key_len bytes                                     */
    uint8_t *end_kinds;       /* 0 = Unbounded, 1 = Excluded(key)                        */
    void *end_keys;           /* cap * key_len bytes                                     */
    rh_aggregate *aggregates; /* the segment's aggregate (unused for enumerations)       */
    size_t n;                 /* items                                                   */
    size_t cap;               /* capacity of the arrays (>= n)                           */
} rh_segments;
typedef struct rh_round_outcome { /* RoundOutcome (protocol.rs:135-142)                 */
    uint64_t skipped, enumerated, split, children, dropped_malformed;
} rh_round_outcome;
int rh_store_protocol_round(rh_store *store, int policy, uint64_t fan_out, const rh_segments *active,
                            rh_segments *children, rh_segments *enumerations, rh_round_outcome *outcome);

/* Host tier (the diff path is latency-bound).  enable = 1 keeps, next to the
 * HBM-resident store, a host copy of the keys in rank order and the exclusive prefix sums of the
 * per-row fingerprints (computed on the device from the GPU lift; (key_len + 32) B of page-locked
 * host memory per row), refreshed on the first question after the contents change.  Then
 * rank / ranks / select / keys, aggregate(s) by rank or by key bounds, resolve / split with at most
 * 16 * round_max questions, and protocol rounds of at most round_max segments are answered on the
 * host: no device round trip, O(log n) per question -- the reference's query cost
 * (query.rs:25-167).  Larger rounds stay on the device.  round_max 0 = the default (128).
 * enable = 0 frees the copy.  Answers are identical either way.                              */
int rh_store_set_host_tier(rh_store *store, int enable, uint64_t round_max);
/* The tier after a batch (host_tier.hpp, host_delta.hpp): the tier holds a copy of the device's
 * base run plus a B+ tree of the signed deltas of every batch since (the device's own DeltaRecs,
 * count and contribution per touched key), so a batch of up to max(2^16, min(base / 8, 2^18)) rows
 * updates it in O(batch log n) -- the reference's O(log n) per insert (mutate.rs:23-88).  A
 * larger batch, while the tier's base is still the device's (no compaction since its copy), takes
 * a copy of the device's delta run instead (its DeltaRecs with prefix sums: O(delta run), not
 * O(n)); a load, a batch after a compaction or after such a run copy, or a tree past its size
 * refreshes the base copy: the device compacts and a copy stream brings the new base down into a
 * second page-locked set.  By default (RSOS_HIP_TIER_SYNC unset or 1) the write or load that
 * starts a refresh waits for it, so every question is answered from a fresh tier; with
 * RSOS_HIP_TIER_SYNC=0 writes never wait -- a stale tier hands the questions to the device (which
 * reads base + delta run in place: no question compacts); while the tier's base is still the
 * device's, its refresh is a background copy of the delta run alone (no compaction), taken if
 * nothing was written meanwhile, else a base refresh, into which batches applied during the copy
 * are logged and replayed.  No question waits for an O(n) copy under either policy.
 * Stats (nullable): base rows and delta entries (tree entries + run-copy entries) of a fresh tier
 * (0, 0 when stale), copies taken from the device (base refreshes and run copies) and batch folds
 * so far.
 * Page-locked host memory: enabling the tier (or a reservation) pins (key_len + 32) B per row plus
 * 8 B per 64 rows for the set the tier reads, with 25% headroom; the first refresh after that pins a
 * second set of the same size, which later refreshes alternate with (a failure to pin leaves the
 * tier stale and is never the write's error); the delta run's copy takes ~(key_len + 41) B per
 * delta row (up to a quarter of the rows; two such sets under RSOS_HIP_TIER_SYNC=0, one filled
 * while the tier reads the other).  At 10^8 rows of 16-byte keys: 6 GB, then 12 GB, plus up to
 * 1.4 GB (2.8 GB with writes never waiting).                                                     */
int rh_store_tier_stats(rh_store *store, uint64_t *base_rows, uint64_t *delta_entries, uint64_t *refreshes,
                        uint64_t *folds);
/* Wait until the host tier is fresh (a background refresh landed and swapped in, one started if
 * none was under way): a warm store for benchmarks and tests.  No-op with the tier off.          */
int rh_store_tier_sync(rh_store *store);
/* The refresh policy of one store (its default: RSOS_HIP_TIER_SYNC when the store was created,
 * else 1).  keep_fresh = 1: a write, load or reservation that needs the tier copied again waits
 * for the copy, so every question is answered on the host; 0: writes never wait for a copy, and
 * questions go to the device while one is in flight.  Takes effect from the next write; a copy in
 * flight is waited for first.                                                                  */
int rh_store_set_tier_policy(rh_store *store, int keep_fresh);

/* Staged single-record updates: Rsos::insert / delete one record at a time (mutate.rs:23-154)
 * without one device round trip each.  rh_store_stage appends m host rows (columns as for
 * rh_store_apply; ops[i] 0 = insert-or-overwrite, 1 = delete) to the store's pending batch and
 * returns; the next call that reads the store (len, aggregate*, rank*, select, keys, rounds,
 * stats, compact, apply, ...) first applies the pending rows as ONE batch, so every answer sees
 * every staged record (one-snapshot-per-round, rbsr/src/rsos_view.rs:36).  A key staged more
 * than once keeps its last operation, exactly as applying them in order would.  A load or
 * snapshot reload drops the pending rows (it replaces the contents).  A staged batch the store
 * rejects is dropped and its error returned by the call that flushed it.                      */
int rh_store_stage(rh_store *store, const rh_columns *host_cols, const uint8_t *ops, size_t m);

/* Batched insert / overwrite / delete (FingerprintTreeMap::insert / remove, mutate.rs:23-154).
 * ops[i]: 0 = insert-or-overwrite record i, 1 = delete key i (its value columns are ignored).
 * Keys within one batch must be distinct (RH_ERR_ARG, store unchanged).  On return every
 * aggregate reflects the whole batch; an overwrite replaces the element's fingerprint (the
 * `new - old` delta of mutate.rs:31-41), so re-delivering a record changes nothing.
 * n_new / n_overwritten / n_deleted (nullable) report what happened.
 * _device: columns and ops already in HBM (the on-GPU incremental update of config 5).    */
int rh_store_apply(rh_store *store, const rh_columns *host_cols, const uint8_t *ops, size_t n,
                   uint64_t *n_new, uint64_t *n_overwritten, uint64_t *n_deleted);
int rh_store_apply_device(rh_store *store, const rh_columns *dev_cols, const uint8_t *dev_ops, size_t n,
                          uint64_t *n_new, uint64_t *n_overwritten, uint64_t *n_deleted, void *after_stream);
/* k device batches applied in order, each exactly as rh_store_apply_device would apply it
 * (dev_ops: k pointers, or NULL for all-insert batches; an entry may be NULL too).  Batch i + 1
 * is key-sorted while the host waits for batch i's result, so queued batches keep the device busy
 * (a replica's write path draining several received batches).  counts (nullable): 3 per batch,
 * new / overwritten / deleted.  On an error the batches before the failing one stay applied.   */
int rh_store_apply_device_many(rh_store *store, const rh_columns *dev_cols, const uint8_t *const *dev_ops,
                               const size_t *n, size_t k, uint64_t *counts, void *after_stream);

/* LSM maintenance.  A batch merges into a sorted signed-delta run (O(batch + delta)); the delta
 * run merges into the base run when it exceeds max(base / divisor, min_rows) rows (default
 * 6, 65536), and before a fingerprint dump or a key dump of more than 2^22 rows.  Every other
 * read -- rank / select / keys, aggregates by rank or by key, resolve / split and protocol rounds --
 * reads base + delta run in place (select over both through the run's count prefix), so no read
 * pays an O(n) merge.  Results never depend on the policy, only timings do.               */
int rh_store_compact(rh_store *store);
int rh_store_set_compaction(rh_store *store, uint64_t divisor, uint64_t min_rows);
/* Capacity for `rows` resident rows fed batches of up to `batch_rows` rows (the device-side
 * analogue of reserving a collection's capacity): both run buffers, the batch buffers and the
 * merge scratch are sized up front, so later batches and compactions never reallocate (a
 * reallocation frees the old buffer, and hipFree waits for the whole device).  Compacts first;
 * contents and every answer are unchanged.  Optional: buffers otherwise grow on demand.    */
int rh_store_reserve(rh_store *store, uint64_t rows, uint64_t batch_rows);
int rh_store_stats(rh_store *store, uint64_t *base_rows, uint64_t *delta_rows, uint64_t *compactions);
/* Which batch path ran (nullable outputs): batches of up to 1,024 rows (512 for 32-byte keys) take
 * the small-batch path -- one workgroup sorts, lifts and searches them and forms their deltas, then
 * one merge launch, the rows and the results read and written in place in page-locked host memory
 * (a replica's network merge, src/replica/dispatch.rs:188-196); larger ones the large-batch path.
 * Env RSOS_HIP_SMALL_MAX=<rows> (read when a store is created) caps the small path; 0 turns it off. */
int rh_store_batch_stats(rh_store *store, uint64_t *small_batches, uint64_t *large_batches);

/* ---- snapshot reload ------------------------------------------------------------------
 * FileSnapshot (src/snapshot.rs:30-58): "RCNL", u32 LE format version 1, then bincode 1.3.3
 * (fixint, LE) of PersistedState<K, V> (lww-register/src/persistence.rs:62-70), whose first
 * field is entries: Vec<(K, Entry<Timestamp, V>)> (:32).  Reload replays the entries through
 * just_insert_bulk (src/replicated_map/persistence.rs:143): every entry goes into the dated map
 * and its projection (src/replica/write.rs:26-46,107-121), in file order, so a repeated key keeps
 * its last entry.  The entries are located and decoded on the device; PersistedState.members
 * and .tombstone_acks follow them at entries_end and stay with the host.
 * Keys in the file: u32 / u64 as fixed LE; byte keys as [u8; L] (RH_FORM_ARRAY, a bincode tuple:
 * the raw bytes) or Vec<u8> / String (RH_FORM_VEC: u64 length L, then the bytes).  Values of
 * kind BYTES are Vec<u8> (u64 length, then the bytes).  Key and value lengths must be
 * multiples of 4 (RH_ERR_UNSUPPORTED otherwise).                                            */
typedef enum rh_key_form { RH_FORM_ARRAY = 0, RH_FORM_VEC = 1 } rh_key_form;

typedef struct rh_snapshot_info {
    uint64_t entries;     /* PersistedState.entries.len()                                  */
    uint64_t tombstones;  /* entries holding State::Tombstone                               */
    uint64_t entries_end; /* file offset of PersistedState.members (just past the entries)  */
    uint64_t keys;        /* distinct keys loaded (< entries when a key repeats)            */
} rh_snapshot_info;

/* Check the 8-byte header (magic, version) and read the entry count; host bytes, len >= 16.
 * RH_ERR_DATA with the reference's message on a short file, wrong magic or version.        */
int rh_snapshot_header(const void *bytes, size_t len, uint64_t *entries);
/* Decode the entries of a device-resident snapshot into device columns with room for `cap`
 * rows.  keys / phys / logical / node / tags / values are all written (a tombstone's value
 * row is zero-filled; tags = the State variant).  Synchronous on `stream`.                */
int rh_snapshot_decode_device(const rh_schema *schema, int key_form, const void *dev_bytes, size_t len,
                              const rh_columns *dev_out, size_t cap, rh_snapshot_info *info, void *stream);
/* Reload: replace the contents of `dated` (record_kind DATED) and / or `projection`
 * (PROJECTION) with a snapshot's entries; either store may be NULL, and both must have the
 * same key and value kinds on the same device.  bytes_on_device: 0 = host bytes (copied to
 * the device), 1 = device bytes (written on `after_stream`, which the store waits for).
 * info (nullable) reports what was read.                                                   */
int rh_store_load_snapshot(rh_store *dated, rh_store *projection, int key_form, const void *bytes, size_t len,
                           int bytes_on_device, rh_snapshot_info *info, void *after_stream);

/* ---- RangeAggregate wire codec ---------------------------------------------------------
 * RangeAggregate<K> (rbsr/src/protocol.rs:63-88) under the gossip codec: bincode 1.3.3
 * DefaultOptions, i.e. varint integers (gossip/src/bincode.rs:65-70; golden vector
 * tests/wire_format.rs:37-62).  Per item: start bound (varint tag 0 = Unbounded,
 * 1 = Included, then the key), end bound (0 = Unbounded, 1 = Excluded, then the key), the 32
 * fingerprint bytes (rsos/src/fingerprint.rs:74-83), the size as a varint.  Keys: u32 / u64
 * varint, [u8; L] raw bytes (RH_FORM_ARRAY), Vec<u8> varint length + bytes (RH_FORM_VEC).
 * msg_tag >= 0 prefixes every item with that Message variant (0 = ComparisonItem,
 * 3 = ValueComparisonItem, src/replica.rs:184-199), giving the byte stream send_messages_to
 * packs into datagrams (src/replica/pacing.rs:200); msg_tag = -1 encodes bare items.
 * Bound kinds are arrays of r bytes; keys are r * key_len bytes (rows of unbounded sides are
 * ignored on encode and zeroed on decode).                                                 */
/* out == NULL: only *out_len = the encoded length.  RH_ERR_ARG if cap < that length.      */
int rh_wire_encode_range_aggregates(const rh_schema *schema, int key_form, int msg_tag, const uint8_t *start_kinds,
                                    const void *start_keys, const uint8_t *end_kinds, const void *end_keys,
                                    const rh_aggregate *aggregates, size_t r, uint8_t *out, size_t cap,
                                    size_t *out_len);
/* Decode items until the input ends or r_cap items are read (gossip::bincode::decode_stream,
 * gossip/src/bincode.rs:79-100); *r_out items, *consumed bytes.  RH_ERR_DATA on malformed
 * bytes (unknown tag, bad varint, truncated item, Vec length != key_len).                  */
int rh_wire_decode_range_aggregates(const rh_schema *schema, int key_form, int msg_tag, const uint8_t *in, size_t len,
                                    size_t r_cap, uint8_t *start_kinds, void *start_keys, uint8_t *end_kinds,
                                    void *end_keys, rh_aggregate *aggregates, size_t *r_out, size_t *consumed);

/* ---- the encoded store: Rsos<K> for any serde K / V -------------------------------------------
 * For keys and values without a fixed-width column form (ReplicatedMap<String, String>,
 * examples/k8s/main.rs:53; Vec<u8>, structs).  A record is its canonical bytes:
 * rsos::encoding::encode_to_vec(&k) followed by encode_to_vec(&v) (public-api/rsos.txt:61) --
 * lift(k, v) is BLAKE3 of exactly that concatenation (rsos/src/fingerprint.rs:270-275) -- hashed on
 * the device on ingest.  The caller keeps the keys and their order (the key type's Ord: for
 * String / Vec<u8> not the order of their length-prefixed encodings) and addresses rows by rank;
 * the device keeps the fingerprints in rank order with the block / super-block sums.  Record i's
 * bytes are bytes[offsets[i] .. offsets[i + 1]) (host buffers; offsets non-decreasing).
 * load: n records in key order, duplicates removed by the caller.
 * apply: m rank-addressed ops against the current order, sorted by position -- kind 0 inserts a
 *   record before the row now at pos (pos <= size), 1 overwrites row pos, 2 deletes row pos; at
 *   one position the inserts come first, then at most one overwrite or delete.  Ops 0 and 1 take
 *   the batch's records in order (nrec of them).  RH_ERR_ARG leaves the store unchanged.
 * aggregates: over rank ranges [lo, hi) (clamped; inverted = ZERO), from the host tier's prefix
 *   sums when it is on (rh_estore_set_host_tier), else one device launch.                     */
typedef struct rh_estore rh_estore;
int rh_estore_create(int device, rh_estore **out);
int rh_estore_destroy(rh_estore *store);
int rh_estore_load(rh_estore *store, const uint8_t *bytes, const uint64_t *offsets, size_t n);
int rh_estore_apply(rh_estore *store, const uint64_t *pos, const uint8_t *kinds, size_t m, const uint8_t *bytes,
                    const uint64_t *offsets, size_t nrec);
int rh_estore_len(rh_estore *store, uint64_t *out);
int rh_estore_root(rh_estore *store, rh_aggregate *out);
int rh_estore_aggregates(rh_estore *store, const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out);
int rh_estore_fingerprints(rh_estore *store, uint64_t lo, uint64_t hi, uint8_t *host_out);
int rh_estore_set_host_tier(rh_estore *store, int enable);

/* ---- the sharded store: one map over several GPUs ------------------------------------------
 * The north_star's key-range shards inside one replica (a replica is one process
 * holding one map, src/replica.rs:68-74): rh_sstore is n column stores, shard s on devices[s]
 * (a device may repeat), shard s holding the keys in [split[s - 1], split[s]).  Same schema rules,
 * same answers, same errors as one rh_store holding the whole map -- the Rsos<K> surface
 * (rsos/src/rsos_trait.rs:39-90) and the protocol round (rbsr/src/protocol.rs:212-317).  Every
 * question is decomposed over the shards with no device-to-device traffic (ranks and aggregates
 * add over a key-range partition, aggregate.rs:79-89; select goes to the shard holding its rank;
 * a round's segments inside one shard's range are that shard's own round, a segment straddling a
 * boundary is resolved from its two boundary shards and cut on the host), and the shards are
 * driven concurrently by host threads (one per shard; at most 4 per device when shards share
 * one, RSOS_HIP_SSTORE_GROUP overriding).  Every call is synchronous and takes the map's
 * lock: each answer is one snapshot of every shard (rbsr/src/rsos_view.rs:36).
 * Splitters: until the first load the key space is cut evenly (u32 / u64 keys at multiples of
 * 2^32 / n and 2^64 / n, byte keys by their leading 8 bytes), so single inserts spread over the
 * shards; a load cuts its rows at equal counts (shard s gets rows [n_rows * s / n, n_rows * (s + 1) / n)).
 * apply: a batch with a repeated key is rejected (RH_ERR_ARG) before any shard changes.
 * Round outputs belong to the sharded store (valid until its next call), as rh_store_protocol_round's.
 * reserve: each shard reserves rows / n (+ 1/8) resident rows and batches of batch_rows.        */
typedef struct rh_sstore rh_sstore;
int rh_sstore_create(const int *devices, int n, const rh_schema *schema, rh_sstore **out);
int rh_sstore_destroy(rh_sstore *store);
int rh_sstore_shard_count(rh_sstore *store);
/* shard i's store (borrowed: stats, tier stats; destroyed with the sharded store)            */
int rh_sstore_shard(rh_sstore *store, int i, rh_store **out);
/* the n - 1 splitters (key_len bytes each); set_splitters only while the map is empty
 * (RH_ERR_STATE otherwise), non-decreasing                                                    */
int rh_sstore_splitters(rh_sstore *store, void *out);
int rh_sstore_set_splitters(rh_sstore *store, const void *keys);
int rh_sstore_load(rh_sstore *store, const rh_columns *host_cols, size_t n);
int rh_sstore_stage(rh_sstore *store, const rh_columns *host_cols, const uint8_t *ops, size_t m);
int rh_sstore_apply(rh_sstore *store, const rh_columns *host_cols, const uint8_t *ops, size_t n, uint64_t *n_new,
                    uint64_t *n_overwritten, uint64_t *n_deleted);
int rh_sstore_len(rh_sstore *store, uint64_t *out);
int rh_sstore_aggregates(rh_sstore *store, const uint64_t *lo, const uint64_t *hi, size_t r, rh_aggregate *out);
int rh_sstore_aggregate_keys(rh_sstore *store, int lo_kind, const void *lo_key, int hi_kind, const void *hi_key,
                             rh_aggregate *out);
int rh_sstore_rank(rh_sstore *store, const void *key, uint64_t *out);
int rh_sstore_ranks(rh_sstore *store, const void *keys, size_t m, uint64_t *out);
int rh_sstore_select(rh_sstore *store, uint64_t r, void *key_out);
int rh_sstore_keys(rh_sstore *store, uint64_t lo, uint64_t hi, void *host_out);
int rh_sstore_fingerprints(rh_sstore *store, uint64_t lo, uint64_t hi, uint8_t *host_out);
int rh_sstore_resolve_segments(rh_sstore *store, size_t r, const uint8_t *start_kinds, const void *start_keys,
                               const uint8_t *end_kinds, const void *end_keys, uint64_t *raw_start,
                               uint64_t *raw_end, rh_aggregate *local);
int rh_sstore_split_segments(rh_sstore *store, size_t m, const uint64_t *select_ranks, void *keys_out, size_t q,
                             const uint64_t *lo, const uint64_t *hi, rh_aggregate *out);
int rh_sstore_protocol_round(rh_sstore *store, int policy, uint64_t fan_out, const rh_segments *active,
                             rh_segments *children, rh_segments *enumerations, rh_round_outcome *outcome);
int rh_sstore_set_host_tier(rh_sstore *store, int enable, uint64_t round_max);
int rh_sstore_set_tier_policy(rh_sstore *store, int keep_fresh);
int rh_sstore_reserve(rh_sstore *store, uint64_t rows, uint64_t batch_rows);
int rh_sstore_compact(rh_sstore *store);

/* ---- testing ---------------------------------------------------------------------------
 * Make the named internal failure point fail once (RH_ERR_OOM) on the calling thread; NULL or
 * "" clears it.  Points: "snapshot.load_begin" (the projection store's half of a reload),
 * "snapshot.load_finish" (the dated store's), "tier.run_copy" (the host tier's copy of the delta
 * run after a large batch: the batch still succeeds, the tier goes stale), "small_batch.merge"
 * (the next small batch's delta merge is reported failed when the store is next entered: that call
 * and every later one return RH_ERR_HIP naming it, until a load replaces the contents),
 * "sstore.apply_last_shard" (a sharded apply's last shard).  Three points instead make the next
 * launch waited for through a sequence word find that word already holding the number it will
 * store, as a reused buffer may: "round.stale_seq" (a one-launch device round), "query.stale_seq"
 * (a one-launch device rank / select / aggregate), "small_batch.stale_seq" (a small batch); the
 * answer must not change.  For tests only.                                                   */
int rh_debug_fail_point(const char *name);

/* ---- measurement -----------------------------------------------------------------------
 * on != 0: time every following snapshot reload's two device stages with HIP events on the
 * loading store's stream; rh_debug_last_reload_us reads the last reload's times back in
 * microseconds: locate = the entry walk and the transfer-function tree, lift = the fused pass
 * (listing, both lifts, keys, samples and block sums; snapshot reloads of records up to 192 B).
 * Both are 0 until a timed reload has run.                                                  */
int rh_debug_reload_timing(int on);
int rh_debug_last_reload_us(double *locate_us, double *lift_us);
/* on != 0: time every following large batch's fused lift + search launch (k_lift_search, the
 * batch path's dominant kernel) with HIP events on the store's stream, accumulated over every
 * store; rh_debug_batch_kernel_us reads the sum (microseconds) and the number of timed launches,
 * on = 1 also zeroes them.                                                                     */
int rh_debug_batch_timing(int on);
int rh_debug_batch_kernel_us(double *lift_search_us, uint64_t *launches);

#ifdef __cplusplus
}
#endif
#endif /* RSOS_HIP_H */
