/* hga.h — C ABI of the MI355X k-mer hot path (libhga.so).
 *
 * The reference has no FFI; its seams are a process boundary and an in-process C++
 * API.  Every entry point below names the reference interface it replaces
 * (paths relative to the reference tree).  Plain pointers and sizes only; no
 * exception crosses the ABI; every call returns an hga_status and
 * hga_last_error() returns a thread-local message for the last failure.
 *
 * Threading: one hga_ctx owns one HIP stream on one device.  A ctx is not
 * thread-safe; several ctx per device are allowed.  Host buffers passed in are
 * caller-owned and may be freed as soon as the call returns.  Buffers the library
 * allocates for the caller are released with hga_free().
 */
#ifndef HGA_H
#define HGA_H

#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct hga_ctx hga_ctx;

typedef enum hga_status {
    HGA_OK = 0,
    HGA_ERR_INVALID = 1, /* bad argument (k out of range, unknown file index, ...)  */
    HGA_ERR_HIP = 2,     /* a HIP runtime call failed                                */
    HGA_ERR_OOM = 3,     /* device or host allocation failed                         */
    HGA_ERR_STATE = 4,   /* call out of order (e.g. select before count_run)         */
    HGA_ERR_COMM = 5     /* RCCL failure                                             */
} hga_status;

/* Thread-local text of the last error ("" if none). */
const char* hga_last_error(void);
/* Frees any buffer the library returned through an out-pointer. */
void hga_free(void* p);
/* Number of visible HIP devices. */
hga_status hga_device_count(int* n);
/* Library/kernel build identification string (static). */
const char* hga_version(void);

hga_status hga_ctx_create(hga_ctx** out, int device);
hga_status hga_ctx_destroy(hga_ctx* ctx);

/* ------------------------------------------------------------------------------
 * Counting — replaces reference seam #1 (the per-file
 *   popen("./occurrences/run_jellyfish.sh <reads> <k> <sorted>")  of
 *   src/occurrences/JellyfishOccurrenceReader.cpp:19-24, i.e. `jellyfish bc/count -C
 *   --bc`, `dump -c` and `LC_ALL=C sort`, src/occurrences/run_jellyfish.sh:3-6)
 * and both k-way merge passes of seam #2 (JellyfishOccurrenceReader::get_next_kmer,
 *   get_specificity, export_kmers; src/occurrences/JellyfishOccurrenceReader.cpp:63-135).
 * ------------------------------------------------------------------------------ */

/* Starts a counting session: k in [1,32], n_files >= 1 (one file = one haplotype,
 * README.md:36).  Replaces JellyfishOccurrenceReader(paths, k)
 * (src/occurrences/JellyfishOccurrenceReader.h:32). */
hga_status hga_count_begin(hga_ctx* ctx, int k, uint32_t n_files);

/* Appends sequence bytes of file `file` (copied to HBM).  `seq` holds whole reads
 * separated by any byte that is not A/C/G/T (either case), e.g. '\n'; windows
 * containing such a byte are not counted (jellyfish semantics).  May be called
 * several times per file; a read must not straddle two calls. */
hga_status hga_count_add(hga_ctx* ctx, uint32_t file, const char* seq, uint64_t n_bytes);

/* Adds file `file`'s rows from an existing "<reads>_<k>-mers_sorted" dump instead of its
 * reads: the reference skips jellyfish for a file whose dump exists and merges the dump
 * verbatim (src/occurrences/JellyfishOccurrenceReader.cpp:19-24 and the reader's
 * get_next_kmer, :63-86).  keys = canonical codes (< 4^k, any order), counts >= 1
 * (rows with count 0 are ignored); copied, may be freed on return.  hga_count_run then
 * counts the files given by reads (with the per-file drop) and sums in the dump rows
 * without dropping any.  A file may have both reads and rows; their counts add. */
hga_status hga_count_add_rows(hga_ctx* ctx, uint32_t file, const uint64_t* keys, const uint32_t* counts,
                              uint64_t n);

/* Runs the device pipeline on everything added: canonical k-mers, per-file exact
 * counts, per-file drop of k-mers whose count is < min_per_file (2 = jellyfish
 * `--bc`), merge across files.  May be re-run (bench).  Asynchronous: the launches are
 * queued and the call returns; the run's own failures (level-1 pool, unsplittable bucket,
 * row capacity) are reported by the next count call that consumes its rows
 * (hga_count_spec_hist, _select*, _rows, _dump, _get_stats, the exchange calls), which
 * then fails with that status.  A run nobody consumed is discarded, errors included, by the
 * next hga_count_run or hga_count_add_rows (whose rows replace it). */
hga_status hga_count_run(hga_ctx* ctx, uint32_t min_per_file);

typedef struct hga_count_stats {
    uint64_t instances;      /* k-mer windows counted (all files)                  */
    uint64_t distinct_rows;  /* merged rows present after the per-file drop       */
    uint64_t bytes;          /* sequence bytes resident on the device              */
    uint32_t buckets;        /* hash buckets used by the binning pass              */
    uint32_t max_split;      /* largest sub-pass split any bucket needed           */
} hga_count_stats;
hga_status hga_count_get_stats(hga_ctx* ctx, hga_count_stats* out);

/* Specificity histogram — JellyfishOccurrenceReader::get_specificity
 * (src/occurrences/JellyfishOccurrenceReader.cpp:88-108): for every merged row,
 * spec = first threshold > ((double)max_f c_f / (double)Σ c_f) * 100 and
 * result[spec][Σc] += 1.  thr must be ascending; every row must fall below the last
 * threshold.  Output: *triples = malloc'ed int64 [3 * *n]: (threshold index, total,
 * unique k-mer count), ordered by threshold then total (std::map order);
 * thresholds with no rows produce no triple. */
hga_status hga_count_spec_hist(hga_ctx* ctx, const double* thr, uint32_t n_thr,
                               int64_t** triples, uint64_t* n);

/* Export selection — JellyfishOccurrenceReader::export_kmers
 * (src/occurrences/JellyfishOccurrenceReader.cpp:110-135) with percent >= 1: the
 * canonical codes of all merged rows with lower <= Σc <= upper, ascending
 * (== the reference's LC_ALL=C string order for fixed k), and the number of them
 * present in exactly one file (:128-130).  *keys malloc'ed (hga_free).
 * Sampling for percent < 1 is host work on this output (see host/jf_occurrences). */
hga_status hga_count_select(hga_ctx* ctx, int64_t lower, int64_t upper, uint64_t** keys,
                            uint64_t* n, uint64_t* n_discriminative);
/* Same, plus one byte per key: 1 if that k-mer is present in exactly one file.  The
 * host needs the flags when it samples with percent < 1 (:128-130).  *keys and
 * *discriminative are malloc'ed (hga_free). */
hga_status hga_count_select_ex(hga_ctx* ctx, int64_t lower, int64_t upper, uint64_t** keys,
                               uint8_t** discriminative, uint64_t* n, uint64_t* n_discriminative);
/* Same, leaving the sorted keys on the device (bench / chained use). */
hga_status hga_count_select_device(hga_ctx* ctx, int64_t lower, int64_t upper,
                                   uint64_t* n, uint64_t* n_discriminative);

/* All merged rows, ascending by code: keys[rows], counts[rows * n_files] row-major.
 * This is the stream JellyfishOccurrenceReader::get_next_kmer yields. */
hga_status hga_count_rows(hga_ctx* ctx, uint64_t** keys, uint32_t** counts, uint64_t* rows);

/* One file's dump: rows with count >= min_per_file in that file, ascending — the
 * content of "<reads>_<k>-mers_sorted" (run_jellyfish.sh:5-6). */
hga_status hga_count_dump(hga_ctx* ctx, uint32_t file, uint64_t** keys, uint32_t** counts,
                          uint64_t* rows);

/* Multi-GPU owner exchange (the reference is single-process).  Each rank
 * counts its shard with hga_count_run(ctx, 1), so no per-file singleton is dropped before
 * the global sum, then:
 *   hga_count_partition  writes the rank's merged rows grouped by owner into caller-owned
 *     DEVICE buffers keys_out[rows] and counts_out[rows * n_files] (row-major), owner o first
 *     covering codes in [splitters[o-1], splitters[o]) (n_owners-1 ascending splitters, host
 *     memory); rows_per_owner[n_owners] (host) receives each owner's slice length.  The
 *     buffers hold hga_count_get_stats().distinct_rows rows.  Returns when they are complete.
 *   (caller) one all-to-all per array over RCCL.
 *   hga_count_merge      takes the rows received by this owner (DEVICE pointers, any order,
 *     at most one row per key per source rank), sums equal keys, applies the per-file drop
 *     (count >= min_per_file, the `--bc` of run_jellyfish.sh:3-6) and makes the result the
 *     ctx's merged rows: spec_hist / select / rows / dump then run on this owner's key range,
 *     ascending, exactly as JellyfishOccurrenceReader.cpp:63-135 would over the whole input. */
hga_status hga_count_partition(hga_ctx* ctx, const uint64_t* splitters, uint32_t n_owners,
                               uint64_t* keys_out, uint32_t* counts_out, uint64_t* rows_per_owner);
hga_status hga_count_merge(hga_ctx* ctx, const uint64_t* keys, const uint32_t* counts, uint64_t n,
                           uint32_t min_per_file);

/* Packed form of the same exchange (half the bytes): one u64 per row piece, key in the low 2k
 * bits, file f's count in the `bits` bits above it (bits = (64 - 2k) / n_files, 0 when below 4
 * or n_files > 8: use the wide form).  A row whose count exceeds 2^bits - 1 is sent as several
 * pieces with the same key; the owner's merge sums them.
 *   hga_count_partition_packed: pieces grouped by owner into DEVICE buffer out[capacity];
 *     pieces_per_owner[n_owners] and *total (host).  If *total > capacity nothing is written
 *     and HGA_ERR_OOM is returned (call again with room for *total).
 *   hga_count_merge_packed: the pieces this owner received (DEVICE pointer, any order). */
hga_status hga_count_pack_bits(hga_ctx* ctx, int* bits);
hga_status hga_count_partition_packed(hga_ctx* ctx, const uint64_t* splitters, uint32_t n_owners,
                                      uint64_t* out, uint64_t capacity, uint64_t* pieces_per_owner,
                                      uint64_t* total);
hga_status hga_count_merge_packed(hga_ctx* ctx, const uint64_t* pieces, uint64_t n,
                                  uint32_t min_per_file);

/* ------------------------------------------------------------------------------
 * Multi-GPU counting inside the library (SURVEY.md §8(b) `hga_comm_init`, §8(e)).  The
 * reference is single-process; this replaces its one jellyfish run per file with one rank per
 * GPU, each counting a contiguous shard of every file.  One hga_ctx per rank: one process per
 * GPU, or one thread per GPU in one process (bin/jf_occurrences --gpus N).
 *
 *   every rank:  hga_count_begin / hga_count_add (its shard) / hga_count_run(ctx, 1)
 *                hga_count_exchange(ctx, min_per_file)   (collective)
 *   then hga_count_spec_hist / _select / _select_ex / _rows / _dump / _get_stats answer for the
 *   whole input, identically on every rank (collectives: call them on every rank, same order);
 *   hga_count_select_device leaves each owner's sorted slice on its device and returns the global
 *   (n, n_discriminative).  Gathered results are the owners' sorted slices merged by key, i.e. the
 *   reference's order (JellyfishOccurrenceReader.cpp:63-135).  A later hga_count_run makes the ctx
 *   local again until the next exchange.  With a communicator attached, hga_count_run(ctx, 1)
 *   already groups its rows for the exchange; local queries before the exchange still work.
 * ------------------------------------------------------------------------------ */
#define HGA_UNIQUE_ID_BYTES 128
/* RCCL unique id (ncclGetUniqueId): create on one rank, hand the bytes to all ranks. */
hga_status hga_comm_unique_id(void* id /* HGA_UNIQUE_ID_BYTES */);
/* RCCL communicator over xGMI for this ctx's device (ncclCommInitRank; blocks until every rank
 * joined).  Exchanges are enqueued on the ctx stream. */
hga_status hga_comm_init(hga_ctx* ctx, const void* unique_id, int rank, int nranks);

/* Host-staged transport supplied by the caller (gloo, MPI, sockets, threads of one process).
 * alltoallv is collective: every rank calls it in the same order; send_bytes[p] bytes at send[p]
 * go to rank p, recv_bytes[p] bytes from rank p land at recv[p] (host memory; the library stages
 * device data).  Returns 0 on success. */
typedef struct hga_transport {
    void* user;
    int (*alltoallv)(void* user, const void* const* send, const uint64_t* send_bytes, void* const* recv,
                     const uint64_t* recv_bytes);
} hga_transport;
hga_status hga_comm_init_host(hga_ctx* ctx, int rank, int nranks, const hga_transport* transport);
/* This ctx's rank and rank count (0 and 1 without a communicator). */
hga_status hga_comm_info(hga_ctx* ctx, int* rank, int* nranks);
/* Gathered lists on one rank only (the export and the dumps to one writer, as the
 * reference's single export_kmers pass writes them, JellyfishOccurrenceReader.cpp:110-135): after it,
 * hga_count_select / _select_ex / _rows / _dump still run on every rank (collectives), but only rank
 * `root` receives the list; the other ranks get an empty one (*n, *n_discriminative, *rows = 0).  One
 * copy crosses the ranks instead of P.  root = -1 (the default): every rank gets the whole list. */
hga_status hga_comm_set_root(hga_ctx* ctx, int root);
hga_status hga_comm_destroy(hga_ctx* ctx);

/* Owner exchange after hga_count_run(ctx, 1) on every rank: owners hold ranges of a hash of the
 * k-mer; one all-to-all-v of packed row pieces (one u64 each) and one of per-bucket counts, owner
 * merge with the per-file drop count >= min_per_file (jellyfish --bc, run_jellyfish.sh:3-6); rows
 * that do not pack go as (key, counts) rows to canonical-code ranges. */
hga_status hga_count_exchange(hga_ctx* ctx, uint32_t min_per_file);

/* ------------------------------------------------------------------------------
 * SDK lookup — replaces the per-read loop of ReadClusteringEngine::construct_indices
 * (src/clustering/ReadClusteringEngine.cpp:234-299).  The host keeps SDK loading
 * (src/read_clustering.cpp:18-33) and the KmerID assignment (iteration order of the
 * std::unordered_set, ReadClusteringEngine.cpp:237-241).
 * ------------------------------------------------------------------------------ */

/* Uploads the SDK set: keys_in_id_order[i] is the canonical code of KmerID i. */
hga_status hga_lookup_load(hga_ctx* ctx, int k, const uint64_t* keys_in_id_order, uint32_t n);

/* Uploads reads in reader order as a CSR: read i = bases[offsets[i], offsets[i+1]).
 * Read i has ReadID first_read_id + i (SequenceRecordIterator IDs are consecutive,
 * 1-based, src/common/SequenceRecordIterator.cpp:27,168). */
hga_status hga_lookup_set_reads(hga_ctx* ctx, const char* bases, const uint64_t* offsets,
                                uint64_t n_reads, uint32_t first_read_id);

/* Runs the lookup and builds every index on the device. */
hga_status hga_lookup_run(hga_ctx* ctx);

typedef struct hga_lookup_sizes {
    uint64_t n_reads;
    uint64_t windows;   /* k-mer windows scanned                                       */
    uint64_t hits;      /* H: windows whose canonical code is an SDK                   */
    uint64_t firsts;    /* U: distinct (read, KmerID) pairs                            */
    uint64_t reads_hit; /* reads with >= 1 hit (the ReadComponents created)            */
    uint32_t n_sdk;     /* K                                                           */
} hga_lookup_sizes;
hga_status hga_lookup_get_sizes(hga_ctx* ctx, hga_lookup_sizes* out);

/* Caller-allocated output arrays (any may be NULL to skip):
 *  hit_ptr[n+1], hit_kid[H], hit_pos[H]: per read, hits in window order with the
 *      end-exclusive position (KmerIterator::position_in_sequence);
 *  sorted_kid[H]: per read, KmerIDs ascending with duplicates
 *      (ReadComponent::discriminative_kmer_ids, ReadClusteringEngine.cpp:262-272);
 *  first_ptr[n+1], first_kid[U], first_pos[U]: ReadMetaData::kmer_positions
 *      (first occurrence wins, :267) listed by ascending KmerID;
 *  kci_ptr[K+1], kci_read[H]: kmer_component_index, per KmerID the ReadIDs, one per
 *      occurrence, ascending (:262-263, 282-284). */
typedef struct hga_lookup_result {
    uint64_t* hit_ptr;
    uint32_t* hit_kid;
    uint32_t* hit_pos;
    uint32_t* sorted_kid;
    uint64_t* first_ptr;
    uint32_t* first_kid;
    uint32_t* first_pos;
    uint64_t* kci_ptr;
    uint32_t* kci_read;
} hga_lookup_result;
hga_status hga_lookup_fetch(hga_ctx* ctx, const hga_lookup_result* out);

/* Sharded lookup on a ctx with a communicator: every rank loads the same
 * SDK set (hga_lookup_load), sets its contiguous ReadID range of the reads (hga_lookup_set_reads with
 * first_read_id = the range's first ReadID, ranks in ReadID order) and runs hga_lookup_run; then
 * hga_lookup_gather (collective) replaces the ctx's results with the whole input's index, identical
 * on every rank: hga_lookup_get_sizes / hga_lookup_fetch describe all reads in ReadID order, and
 * kmer_component_index is per KmerID the ranks' lists concatenated in rank order (= ascending, as
 * ReadClusteringEngine.cpp:282-284 leaves it).  hga_connections_run then sees every read; each rank
 * passes its own ReadIDs as pivots (categories, if any, for all reads) and hga_connections_gather
 * (collective) joins the ranks' connections in the reference order (score descending, ties by
 * (pivot, candidate); :331) for hga_connections_fetch.  The next hga_lookup_run returns to the rank's
 * own reads. */
hga_status hga_lookup_gather(hga_ctx* ctx);
hga_status hga_connections_gather(hga_ctx* ctx, uint64_t* n);

/* ------------------------------------------------------------------------------
 * HyperLogLog k-mer cardinality — replaces get_approximate_kmer_count
 * (src/occurrences/KmerAnalysis.cpp:15-38), the estimator behind jf_occurrences' automatic
 * k selection (get_unique_k_length, KmerAnalysis.cpp:41-56; src/jellyfish_occurrences.cpp:40-44).
 * ------------------------------------------------------------------------------ */

/* Registers of hll::HyperLogLog(b) (src/lib/HyperLogLog.hpp:96-106) after add() of the
 * canonical code (8 little-endian bytes, MurmurHash3_x86_32 seed 313) of every KmerIterator
 * window of the reads uploaded with hga_lookup_set_reads.  registers[2^b] (caller-allocated)
 * receive M[index] = max rank; order-independent, so bit-identical to the reference.
 * b in [4, 14] (the reference uses 10); k in [1, 32] ("Kmer size is too big" above 32,
 * KmerIterator.cpp:24-26).  The estimate itself is host arithmetic on these registers. */
hga_status hga_hll_registers(hga_ctx* ctx, int k, uint32_t b, uint8_t* registers);

/* ------------------------------------------------------------------------------
 * Connections — ReadClusteringEngine::get_connections / get_all_connections
 * (src/clustering/ReadClusteringEngine.cpp:301-339) on the one-read components that
 * construct_indices leaves (run after hga_lookup_run, on its device-resident indices).
 * For pivot p and every other read c: score = sum over KmerIDs of (occurrences in p) x
 * (occurrences in c), i.e. the robin_map count of :311-315; pairs with score >= min_score
 * are kept (:318-325), the pivot itself never (:316).
 * ------------------------------------------------------------------------------ */

/* pivots: ReadIDs (the reference's component_ids), or NULL for every read with at least
 *   min_kmers hits (min_kmers = 1: get_all_connections, :335-339; min_kmers = s with
 *   min_score = s: the filter_components(... discriminative_kmer_ids.size() >= s) call
 *   site, :750-751).  A pivot without hits yields nothing.
 * categories: per read of the lookup (read order, n_reads), or NULL.  is_good =
 *   categories[p] == categories[c] when given (the reference's debug mode, :319), else 0.
 * Result order: score descending (std::sort(rbegin, rend), :331); ties, unordered in the
 *   reference, by (pivot, candidate) ascending.  *n = number of connections. */
hga_status hga_connections_run(hga_ctx* ctx, const uint32_t* pivots, uint64_t n_pivots, uint32_t min_kmers,
                               uint64_t min_score, const int32_t* categories, uint64_t* n);
/* Copies the result (caller-allocated, n entries each; any may be NULL): ComponentConnection
 * {component_x_id = x, component_y_id = y, score, is_good}
 * (src/clustering/ReadClusteringEngine.h:127-136). */
hga_status hga_connections_fetch(hga_ctx* ctx, uint32_t* x, uint32_t* y, uint64_t* score, uint8_t* is_good);
/* The same for entries [first, first + count) of the result (clipped to n): run_clustering keeps only the
 * first scaffold_forming_fraction of get_all_connections' sorted list (src/clustering/ReadClusteringEngine.cpp:754-755),
 * so the caller fetches just that prefix. */
hga_status hga_connections_fetch_range(hga_ctx* ctx, uint64_t first, uint64_t count, uint32_t* x, uint32_t* y,
                                       uint64_t* score, uint8_t* is_good);

/* ------------------------------------------------------------------------------
 * Measurement: per-kernel device time, recorded with HIP events on the ctx stream.
 * ------------------------------------------------------------------------------ */
hga_status hga_profile_enable(hga_ctx* ctx, int on);
/* Restricts event timing to the comma-separated launch names ("" or NULL = all), so that
 * the untimed launches carry no event overhead. */
hga_status hga_profile_select(hga_ctx* ctx, const char* names);
hga_status hga_profile_reset(hga_ctx* ctx);
/* Total milliseconds and launch count recorded for kernel `name` since the reset. */
hga_status hga_profile_get(hga_ctx* ctx, const char* name, double* ms, uint64_t* launches);
/* Blocks until the ctx stream is idle. */
hga_status hga_sync(hga_ctx* ctx);

#ifdef __cplusplus
}
#endif
#endif /* HGA_H */
