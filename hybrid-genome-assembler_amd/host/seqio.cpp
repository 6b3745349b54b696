// seqio.cpp — see seqio.h.  Reference semantics are cited per function.
#include "seqio.h"
#include "seqio_internal.h"

#include <charconv>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <regex>
#include <stdexcept>
#include <algorithm>
#include <atomic>
#include <thread>

namespace hgah {

std::string FileMeta::repr() const {
    // MetaData::repr (SequenceRecordIterator.h:60-63)
    std::string s = filename + ":\n";
    s += "- " + std::to_string(records) + " reads\n";
    s += "- " + std::to_string(total_bases) + " total bases\n";
    s += "- " + std::to_string(avg_read_length) + " average read length\n";
    s += "- " + std::to_string(max_read_length) + " max read length\n";
    s += "- " + std::to_string(min_read_length) + " min read length\n\n";
    return s;
}

namespace {

enum class Rec { FASTQ, FASTA };
struct EndOfInput {};

// The reader's line stream: getline over the files in order, switching file on EOF.
// Opening a file sniffs its first record to pick the record layout and the header
// parser, then rewinds (load_file_at_position, SequenceRecordIterator.cpp:73-123).
class LineStream {
   public:
    LineStream(const std::vector<std::string>& paths, const HeaderParsers& hp) : paths_(paths), hp_(hp) {}
    int file_index() const { return idx_; }
    Rec rec() const { return rec_; }
    Hdr hdr() const { return hdr_; }
    int file_type() const { return type_; }

    bool open(int pos) {
        if (in_.is_open()) in_.close();
        if (pos >= (int)paths_.size()) return false;
        in_.clear();
        in_.open(paths_[pos]);
        if (!in_) throw std::invalid_argument("File with path \"" + paths_[pos] + "\" does not exist");
        try {
            std::string header = line();
            std::string sequence = line();
            (void)sequence;
            const char h0 = header.empty() ? '\0' : header[0];
            if (h0 == '@') {
                std::string comment = line();
                if (!comment.empty() && comment[0] == '+') { rec_ = Rec::FASTQ; type_ = 1; }
            } else if (h0 == '>') {
                rec_ = Rec::FASTA;
                type_ = 0;
            } else {
                throw std::logic_error("Unrecognized file format");
            }
            if (hp_.parse(Hdr::SIMLORD, header).second != 0) hdr_ = Hdr::SIMLORD;
            if (hp_.parse(Hdr::NANOSIM, header).second != 0) hdr_ = Hdr::NANOSIM;
            if (hp_.parse(Hdr::PASS, header).second != 0) hdr_ = Hdr::PASS;
        } catch (const EndOfInput&) {
            throw std::logic_error("File is empty");
        }
        in_.clear();
        in_.seekg(0, std::ios::beg);
        idx_ = pos;
        return true;
    }

    std::string line() {
        std::string s;
        if (!std::getline(in_, s)) {
            if (open(idx_ + 1)) return line();
            throw EndOfInput{};
        }
        return s;
    }

   private:
    const std::vector<std::string>& paths_;
    const HeaderParsers& hp_;
    std::ifstream in_;
    int idx_ = 0;
    Rec rec_ = Rec::FASTQ;
    Hdr hdr_ = Hdr::UNKNOWN;
    int type_ = 1;
};


}  // namespace

std::string basename_of(const std::string& p) {
    const size_t i = p.find_last_of("/\\");
    return i == std::string::npos ? p : p.substr(i + 1);
}

const HeaderParsers& header_parsers() {
    static const HeaderParsers hp;
    return hp;
}

RecordSet load_records_seq(const std::vector<std::string>& paths, bool annotate, bool keep_text) {
    const HeaderParsers& hp = header_parsers();
    LineStream ls(paths, hp);
    RecordSet rs;
    rs.file_meta.resize(paths.size());
    if (!paths.empty()) ls.open(0);
    int prev_file = -1;
    std::vector<std::string> names;
    FileMeta* cur = nullptr;
    uint64_t sum_all = 0;
    while (true) {
        std::string header, seq, qual;
        try {   // read_fastq_record / read_fasta_record (SequenceRecordIterator.cpp:137-153)
            if (ls.rec() == Rec::FASTQ) {
                header = ls.line();
                seq = ls.line();
                (void)ls.line();
                qual = ls.line();
            } else {
                header = ls.line();
                seq = ls.line();
            }
        } catch (const EndOfInput&) {
            break;
        }
        const int fidx = ls.file_index();
        const std::string hdr = header.empty() ? std::string() : header.substr(1);
        const auto se = hp.parse(ls.hdr(), hdr);
        rs.bases.append(seq.data(), seq.size());
        rs.offsets.push_back(rs.bases.size());
        rs.category.push_back(annotate ? fidx : 0);
        rs.start.push_back(se.first != 0 ? se.first : 0);
        rs.end.push_back(se.first != 0 ? se.first + se.second : 0);
        if (keep_text) {
            rs.headers.push_back(hdr);
            rs.qualities.push_back(qual);
        }
        // load_meta_data (SequenceRecordIterator.cpp:31-71)
        if (fidx != prev_file) {
            rs.file_meta[fidx] = FileMeta{};
            rs.file_meta[fidx].filename = basename_of(paths[fidx]);
            rs.file_meta[fidx].file_type = ls.file_type();
            cur = &rs.file_meta[fidx];
            prev_file = fidx;
            names.push_back(cur->filename);
        }
        const uint64_t L = seq.size();
        cur->total_bases += L;
        cur->min_read_length = std::min(cur->min_read_length, L);
        cur->max_read_length = std::max(cur->max_read_length, L);
        cur->records++;
        cur->avg_read_length += L;
        rs.meta.total_bases += L;
        rs.meta.min_read_length = std::min(rs.meta.min_read_length, L);
        rs.meta.records++;
        sum_all += L;
    }
    if (rs.meta.records == 0) throw std::logic_error("No records in the read files");
    rs.meta.avg_read_length = sum_all / rs.meta.records;
    for (size_t i = 0; i < names.size(); ++i) rs.meta.filename += (i ? "__" : "") + names[i];
    for (auto& m : rs.file_meta)
        if (m.records) m.avg_read_length /= m.records;
    rs.categories = annotate ? (uint32_t)rs.file_meta.size() : 1u;
    return rs;
}

Bytes jf_stream_seq(const std::string& path, uint64_t* n_records) {
    std::FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::invalid_argument("File with path \"" + path + "\" does not exist");
    std::string data;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    data.resize(sz > 0 ? (size_t)sz : 0);
    if (sz > 0 && std::fread(&data[0], 1, (size_t)sz, f) != (size_t)sz) {
        std::fclose(f);
        throw std::runtime_error("short read on " + path);
    }
    std::fclose(f);
    Bytes out;
    uint64_t recs = 0;
    size_t i = 0;
    const size_t n = data.size();
    auto next_line = [&](size_t& b, size_t& e) -> bool {
        if (i >= n) return false;
        b = i;
        const void* nl = std::memchr(data.data() + i, '\n', n - i);
        e = nl ? (size_t)((const char*)nl - data.data()) : n;
        i = e < n ? e + 1 : n;
        return true;
    };
    size_t b, e;
    // FASTA: '>' header, sequence lines until the next '>'.  FASTQ: '@' header,
    // sequence lines until a '+' line, then quality lines covering the sequence length.
    bool have = next_line(b, e);
    while (have) {
        if (e == b) { have = next_line(b, e); continue; }
        const char h = data[b];
        if (h == '>') {
            if (recs) out.push_back('\n');
            ++recs;
            while ((have = next_line(b, e)) && !(e > b && data[b] == '>'))
                out.append(data.data() + b, e - b);
        } else if (h == '@') {
            if (recs) out.push_back('\n');
            ++recs;
            size_t seqlen = 0;
            while ((have = next_line(b, e)) && !(e > b && data[b] == '+')) {
                out.append(data.data() + b, e - b);
                seqlen += e - b;
            }
            size_t qlen = 0;
            while (have && qlen < seqlen && (have = next_line(b, e))) qlen += e - b;
            if (have) have = next_line(b, e);
        } else {
            have = next_line(b, e);   // stray line outside a record
        }
    }
    if (n_records) *n_records = recs;
    return out;
}

std::string fmt_double(double v) {
    if (v != v) return "nan";
    if (v == __builtin_inf()) return "inf";
    if (v == -__builtin_inf()) return "-inf";
    char buf[64];
    auto r = std::to_chars(buf, buf + sizeof(buf), v, std::chars_format::scientific);
    std::string sci(buf, r.ptr);
    // sci = [-]d[.ddd]e(+|-)XX
    const size_t epos = sci.find('e');
    const int exp10 = std::stoi(sci.substr(epos + 1));
    if (exp10 < -4 || exp10 >= 16) return sci;   // fmt's exp_lower/exp_upper
    std::string mant = sci.substr(0, epos);
    bool neg = false;
    if (!mant.empty() && mant[0] == '-') { neg = true; mant.erase(0, 1); }
    std::string digits;
    for (char ch : mant)
        if (ch != '.') digits.push_back(ch);
    std::string out;
    const int nd = (int)digits.size();
    const int point = exp10 + 1;   // digits before the decimal point
    if (point <= 0) {
        out = "0." + std::string(-point, '0') + digits;
    } else if (point >= nd) {
        out = digits + std::string(point - nd, '0');
    } else {
        out = digits.substr(0, point) + "." + digits.substr(point);
    }
    if (v == 0.0) out = "0";
    return (neg ? "-" : "") + out;
}

void kmer_to_chars(uint64_t code, int k, char* out) {
    static const char B[4] = {'A', 'C', 'G', 'T'};
    for (int i = k - 1; i >= 0; --i) {
        out[i] = B[code & 3u];
        code >>= 2;
    }
}

std::string kmer_to_string(uint64_t code, int k) {
    std::string s((size_t)k, 'A');
    kmer_to_chars(code, k, &s[0]);
    return s;
}

uint64_t line_canonical(const char* s, size_t len) {
    // KmerIterator(line, k = len).next_kmer(); current_kmer stays 0 when it yields nothing.
    const int k = (int)len;
    if (k < 1) return 0;
    if (k > 32) throw std::invalid_argument("Kmer size is too big");
    const uint64_t mask = k >= 32 ? ~0ull : ((1ull << (2 * k)) - 1);
    uint64_t fwd = 0, rc = 0;
    for (size_t i = 0; i < len; ++i) {
        const char c = s[i];
        uint64_t fc = 0, cc = 0;
        switch (c) {
            case 'A': fc = 0; cc = 3; break;
            case 'C': fc = 1; cc = 2; break;
            case 'G': fc = 2; cc = 1; break;
            case 'T': fc = 3; cc = 0; break;
            default: break;
        }
        fwd = ((fwd << 2) | fc) & mask;
        rc = (rc >> 2) | (cc << (2 * (k - 1)));
    }
    return fwd < rc ? fwd : rc;
}

std::string dump_cache_path(const std::string& reads, int k) {
    return reads + "_" + std::to_string(k) + "-mers_sorted";
}

void read_kmer_dump(const std::string& path, int k, std::vector<uint64_t>& keys, std::vector<uint32_t>& counts) {
    std::FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) throw std::invalid_argument("cannot open k-mer dump " + path);
    std::string data;
    std::fseek(f, 0, SEEK_END);
    const long sz = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    data.resize(sz > 0 ? (size_t)sz : 0);
    const bool ok = sz <= 0 || std::fread(&data[0], 1, (size_t)sz, f) == (size_t)sz;
    std::fclose(f);
    if (!ok) throw std::runtime_error("short read on " + path);
    keys.clear();
    counts.clear();
    const char* p = data.data();
    const char* end = p + data.size();
    uint64_t line_no = 0;
    while (p < end) {
        const char* nl = static_cast<const char*>(std::memchr(p, '\n', (size_t)(end - p)));
        const char* e = nl ? nl : end;
        ++line_no;
        if (e > p) {
            const char* sp = static_cast<const char*>(std::memchr(p, ' ', (size_t)(e - p)));
            if (!sp || sp - p != k)
                throw std::invalid_argument(path + ":" + std::to_string(line_no) + ": expected \"<" +
                                            std::to_string(k) + "-mer> <count>\"");
            uint64_t code = 0;
            for (const char* q = p; q < sp; ++q) {
                uint64_t v;
                switch (*q) {
                    case 'A': v = 0; break;
                    case 'C': v = 1; break;
                    case 'G': v = 2; break;
                    case 'T': v = 3; break;
                    default:
                        throw std::invalid_argument(path + ":" + std::to_string(line_no) + ": non-ACGT k-mer");
                }
                code = (code << 2) | v;
            }
            const char* c = sp;
            while (c < e && *c == ' ') ++c;
            uint32_t cnt = 0;
            auto r = std::from_chars(c, e, cnt);
            if (r.ec != std::errc() || c == e)
                throw std::invalid_argument(path + ":" + std::to_string(line_no) + ": bad count");
            keys.push_back(code);
            counts.push_back(cnt);
        }
        p = nl ? nl + 1 : end;
    }
}

void write_kmer_dump(const std::string& path, int k, const uint64_t* keys, const uint32_t* counts, uint64_t n) {
    write_kmer_dump_rows(path, k, keys, counts, 1, 0, n);
}

void write_kmer_dump_rows(const std::string& path, int k, const uint64_t* keys, const uint32_t* counts, uint32_t F,
                          uint32_t file, uint64_t n) {
    // written to `<path>.tmp` and renamed into place once complete: the cache's existence is all a
    // later run checks (JellyfishOccurrenceReader.cpp:19-24), so an interrupted run (a Ctrl-C at the
    // bounds prompt while the writer thread is busy) must not leave a truncated file under its name
    const std::string tmp = path + ".tmp";
    std::FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) throw std::runtime_error("cannot write " + path);
    // "KMER COUNT\n" lines formatted by host_threads() threads, chunk by chunk in row order, each
    // chunk's text written as soon as it and its predecessors are done
    const uint64_t CH = 1u << 18;   // rows per chunk
    const uint64_t nch = (n + CH - 1) / CH;
    const int T = (int)std::max<uint64_t>(1, std::min<uint64_t>((uint64_t)host_threads(), nch));
    std::vector<std::vector<char>> text(nch);
    std::vector<std::atomic<int>> done(nch);
    for (auto& d : done) d.store(0);
    std::atomic<uint64_t> next{0};
    auto work = [&] {
        char num[16];
        for (uint64_t c; (c = next.fetch_add(1)) < nch;) {
            const uint64_t a = c * CH, b = std::min(n, a + CH);
            std::vector<char>& buf = text[c];
            buf.resize((b - a) * ((size_t)k + 12));
            char* o = buf.data();
            for (uint64_t i = a; i < b; ++i) {
                const uint32_t cnt = counts[i * F + file];
                if (!cnt) continue;   // a row of the merged table without this file
                kmer_to_chars(keys[i], k, o);
                o += k;
                *o++ = ' ';
                auto r = std::to_chars(num, num + sizeof(num), cnt);
                for (const char* q = num; q < r.ptr; ++q) *o++ = *q;
                *o++ = '\n';
            }
            buf.resize((size_t)(o - buf.data()));
            done[c].store(1, std::memory_order_release);
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work);
    bool ok = true;
    if (T == 1) work();
    for (uint64_t c = 0; c < nch; ++c) {   // the writer: chunks in order as they complete
        while (!done[c].load(std::memory_order_acquire)) std::this_thread::yield();
        ok = ok && std::fwrite(text[c].data(), 1, text[c].size(), f) == text[c].size();
        std::vector<char>().swap(text[c]);
    }
    for (auto& x : th) x.join();
    if (std::fclose(f) != 0 || !ok) {
        std::remove(tmp.c_str());
        throw std::runtime_error("cannot write " + path);
    }
    if (std::rename(tmp.c_str(), path.c_str()) != 0) {
        std::remove(tmp.c_str());
        throw std::runtime_error("cannot write " + path);
    }
}

}  // namespace hgah
