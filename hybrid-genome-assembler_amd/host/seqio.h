// seqio.h — host-side sequence input for the two drop-in CLIs.
//
//  * RecordSet / load_records: SequenceRecordIterator semantics
//    (src/common/SequenceRecordIterator.cpp:16-205) for `categorization`: one line
//    stream across all files (std::getline, no CR stripping), FASTQ = 4 lines,
//    FASTA = exactly 2 lines, format sniffed per file, ReadIDs 1-based and
//    continuing across files, category = file index when annotating, simulator
//    header regexes, the metadata pass.
//  * jf_stream: the sequence stream jellyfish reads for the counting path
//    (run_jellyfish.sh:3-4): multi-line FASTA/FASTQ records, sequences joined by
//    '\n' (a non-base byte, so no k-mer window spans two reads).
#pragma once

#include <cstdint>
#include <string>
#include <vector>

namespace hgah {

// Growable byte buffer on anonymous memory (transparent huge pages where the kernel allows),
// never zero-filled: resize() leaves new bytes unspecified.  Holds the readers' large outputs
// (hundreds of MB), where value-initialising a std::string / std::vector costs as much as the
// parse itself.
class Bytes {
   public:
    Bytes() = default;
    ~Bytes();
    Bytes(Bytes&& o) noexcept : p_(o.p_), n_(o.n_), cap_(o.cap_) { o.p_ = nullptr; o.n_ = o.cap_ = 0; }
    Bytes& operator=(Bytes&& o) noexcept;
    Bytes(const Bytes&) = delete;
    Bytes& operator=(const Bytes&) = delete;
    char* data() { return p_; }
    const char* data() const { return p_; }
    size_t size() const { return n_; }
    bool empty() const { return n_ == 0; }
    char& operator[](size_t i) { return p_[i]; }
    char operator[](size_t i) const { return p_[i]; }
    void resize(size_t n);
    void clear() { n_ = 0; }
    void append(const char* s, size_t n);
    void push_back(char c) { append(&c, 1); }
    std::string str() const { return std::string(p_ ? p_ : "", n_); }

   private:
    void reserve(size_t n);
    char* p_ = nullptr;
    size_t n_ = 0, cap_ = 0;
};

struct FileMeta {               // MetaData / ReadFileMetaData, SequenceRecordIterator.h:52-68
    std::string filename;
    uint64_t records = 0;
    uint64_t min_read_length = UINT64_MAX;
    uint64_t max_read_length = 0;
    uint64_t avg_read_length = 0;
    uint64_t total_bases = 0;
    int file_type = 2;          // 0 FASTA, 1 FASTQ, 2 UNKNOWN
    std::string repr() const;   // MetaData::repr, SequenceRecordIterator.h:60-63
};

struct RecordSet {
    // CSR of sequences in reader order; read i has ReadID i + 1.
    Bytes bases;
    std::vector<uint64_t> offsets{0};
    std::vector<int32_t> category;      // GenomeReadData::category_id
    std::vector<uint32_t> start, end;   // simulator-header coordinates (0 when unknown)
    std::vector<std::string> headers;   // without the leading '@' / '>'
    std::vector<std::string> qualities; // empty for FASTA
    std::vector<FileMeta> file_meta;
    FileMeta meta;                      // all files ("__"-joined names)
    uint32_t categories = 1;
    uint64_t size() const { return offsets.size() - 1; }
};

// Throws std::invalid_argument / std::logic_error with the reference's messages.
// keep_text=false skips headers/qualities (the lookup needs sequences only).
// load_records / jf_stream run multi-threaded (fastio.cpp) with host_threads() threads and
// fall back to the sequential *_seq definitions for layouts that are not line-local; the
// results are identical.
RecordSet load_records(const std::vector<std::string>& paths, bool annotate, bool keep_text = true);
RecordSet load_records_seq(const std::vector<std::string>& paths, bool annotate, bool keep_text = true);

// Whole-file read of the sequences jellyfish would count, '\n'-separated.
Bytes jf_stream(const std::string& path, uint64_t* n_records = nullptr);
Bytes jf_stream_seq(const std::string& path, uint64_t* n_records = nullptr);

// Reader threads: set_host_threads(n > 0) overrides HGA_HOST_THREADS (default min(16, cores));
// 1 = the sequential readers.
int host_threads();
void set_host_threads(int n);

// fmt "{}" formatting of a double (shortest round trip, fmt's fixed/exponent switch).
std::string fmt_double(double v);

// KmerIterator::number_to_sequence (src/common/KmerIterator.cpp:44-52).
std::string kmer_to_string(uint64_t code, int k);
void kmer_to_chars(uint64_t code, int k, char* out);

// KmerIterator canonical code of a whole line (load_text_file_kmers, read_clustering.cpp:18-33).
uint64_t line_canonical(const char* s, size_t len);

// load_text_file_kmers (read_clustering.cpp:18-33): the SDK file's canonical codes in KmerID order (the
// iteration order of the std::unordered_set the reference fills line by line,
// ReadClusteringEngine.cpp:237-241); *k = the last line's length.  Lines encoded in parallel; the set's
// order reproduced without building it (unordered_set_order).
std::vector<uint64_t> load_kmer_text(const std::string& path, int* k);
// The iteration order of a libstdc++ std::unordered_set<uint64_t> after inserting keys[0..n) in order.
std::vector<uint64_t> unordered_set_order(const uint64_t* keys, size_t n);

// "<reads>_<k>-mers_sorted" dump cache (JellyfishOccurrenceReader.cpp:19-24; written by
// run_jellyfish.sh:5-6 as `jellyfish dump -c` + LC_ALL=C sort): one "KMER COUNT" line per
// k-mer.  read_kmer_dump parses it like parse_line (JellyfishOccurrenceReader.cpp:9-14); the
// k-mer string is kept as it is (its forward 2-bit code, not re-canonicalised), and a line
// whose k-mer is not k bases of ACGT throws.  write_kmer_dump writes rows in the given order.
void read_kmer_dump(const std::string& path, int k, std::vector<uint64_t>& keys, std::vector<uint32_t>& counts);
void write_kmer_dump(const std::string& path, int k, const uint64_t* keys, const uint32_t* counts, uint64_t n);
// The same from the merged rows (counts row-major [n][F]): the rows with a count in `file`.
void write_kmer_dump_rows(const std::string& path, int k, const uint64_t* keys, const uint32_t* counts, uint32_t F,
                          uint32_t file, uint64_t n);
std::string dump_cache_path(const std::string& reads, int k);   // "{reads}_{k}-mers_sorted"

}  // namespace hgah
