// args.h — the subset of boost::program_options behaviour the two CLIs rely on
// (src/jellyfish_occurrences.cpp:19-31, src/read_clustering.cpp:41-63): positional
// arguments collected into one list, "-x V", "-xV", "--long V", "--long=V", boolean
// switches, and an "unrecognised option" error for anything else.
#pragma once

#include <cstdio>
#include <functional>
#include <map>
#include <stdexcept>
#include <string>
#include <vector>

namespace hgah {

struct ArgSpec {
    std::string longname;   // without "--"
    char shortname;         // 0 if none
    bool is_switch;
    std::string help;
    std::function<void(const std::string&)> set;
};

class ArgParser {
   public:
    void add(const std::string& l, char s, bool sw, const std::string& help,
             std::function<void(const std::string&)> set) {
        specs_.push_back({l, s, sw, help, std::move(set)});
    }
    std::vector<std::string> positional;
    std::map<std::string, int> seen;

    void parse(int argc, char** argv) {
        for (int i = 1; i < argc; ++i) {
            std::string a = argv[i];
            if (a.size() > 2 && a[0] == '-' && a[1] == '-') {
                std::string name = a.substr(2), val;
                const size_t eq = name.find('=');
                bool has_val = eq != std::string::npos;
                if (has_val) { val = name.substr(eq + 1); name = name.substr(0, eq); }
                const ArgSpec* sp = find_long(name);
                if (!sp) throw std::invalid_argument("unrecognised option '--" + name + "'");
                if (!sp->is_switch && !has_val) {
                    if (i + 1 >= argc) throw std::invalid_argument("the required argument for option '--" + name + "' is missing");
                    val = argv[++i];
                }
                apply(*sp, val);
            } else if (a.size() >= 2 && a[0] == '-' && a[1] != '-') {
                const ArgSpec* sp = find_short(a[1]);
                if (!sp) throw std::invalid_argument(std::string("unrecognised option '") + a + "'");
                std::string val;
                if (!sp->is_switch) {
                    if (a.size() > 2) val = a.substr(2);
                    else {
                        if (i + 1 >= argc) throw std::invalid_argument(std::string("the required argument for option '-") + a[1] + "' is missing");
                        val = argv[++i];
                    }
                }
                apply(*sp, val);
            } else {
                positional.push_back(a);
            }
        }
    }
    bool has(const std::string& l) const { return seen.count(l) != 0; }

    std::string describe() const {
        std::string s = "Options:\n";
        for (auto& sp : specs_) {
            std::string left = "  ";
            if (sp.shortname) left += std::string("-") + sp.shortname + " [ --" + sp.longname + " ]";
            else left += "--" + sp.longname;
            if (!sp.is_switch) left += " arg";
            if (left.size() < 40) left += std::string(40 - left.size(), ' ');
            s += left + " " + sp.help + "\n";
        }
        return s;
    }

   private:
    std::vector<ArgSpec> specs_;
    const ArgSpec* find_long(const std::string& n) const {
        for (auto& s : specs_) if (s.longname == n) return &s;
        return nullptr;
    }
    const ArgSpec* find_short(char c) const {
        for (auto& s : specs_) if (s.shortname == c) return &s;
        return nullptr;
    }
    void apply(const ArgSpec& sp, const std::string& v) {
        seen[sp.longname]++;
        if (sp.set) sp.set(sp.is_switch ? std::string("1") : v);
    }
};

}  // namespace hgah
