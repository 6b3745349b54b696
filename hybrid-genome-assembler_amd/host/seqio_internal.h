// seqio_internal.h — pieces shared by the sequential (seqio.cpp) and parallel (fastio.cpp)
// readers.  Not part of any ABI.
#pragma once

#include <cstdint>
#include <regex>
#include <string>
#include <utility>

namespace hgah {

enum class Hdr { UNKNOWN, SIMLORD, NANOSIM, PASS };

struct HeaderParsers {
    // SequenceRecordIterator.h:98-105
    std::regex simlord{";length=([0-9]+)bp;startpos=([0-9]+);"};
    std::regex nanosim{"_([0-9]+)_[^_]+_[^_]+_[^_]+_[^_]+_([0-9]+)_"};
    std::regex pass{"([0-9]+)_([0-9]+)\\|([0-9]+)\\|"};

    // (start, length) as in parse_*_header (SequenceRecordIterator.cpp:179-205)
    std::pair<uint32_t, uint32_t> parse(Hdr h, const std::string& s) const {
        std::smatch m;
        switch (h) {
            case Hdr::SIMLORD:
                if (std::regex_search(s, m, simlord))
                    return {(uint32_t)std::stoul(m[2].str()), (uint32_t)std::stoul(m[1].str())};
                break;
            case Hdr::NANOSIM:
                if (std::regex_search(s, m, nanosim))
                    return {(uint32_t)std::stoul(m[1].str()), (uint32_t)std::stoul(m[2].str())};
                break;
            case Hdr::PASS:
                if (std::regex_search(s, m, pass)) {
                    const uint32_t len = (uint32_t)(std::stoul(m[2].str()) - std::stoul(m[1].str()));
                    return {(uint32_t)std::stoul(m[3].str()), len};
                }
                break;
            default: break;
        }
        return {0, 0};
    }
};

const HeaderParsers& header_parsers();
std::string basename_of(const std::string& p);

}  // namespace hgah
