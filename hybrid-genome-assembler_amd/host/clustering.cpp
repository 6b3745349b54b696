// clustering.cpp — see clustering.h.  Every function cites the reference lines it restates
// (src/clustering/ReadClusteringEngine.cpp unless noted).
#include "clustering.h"

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <cmath>
#include <filesystem>
#include <fstream>
#include <functional>
#include <limits>
#include <memory>
#include <mutex>
#include <queue>
#include <stdexcept>
#include <thread>
#include <unordered_map>

namespace hgah {

void sort_connections(std::vector<Connection>& c) {
    std::sort(c.begin(), c.end(), [](const Connection& a, const Connection& b) {
        if (a.score != b.score) return a.score > b.score;
        if (a.x != b.x) return a.x < b.x;
        return a.y < b.y;
    });
}

namespace {

// timeMeasure / timeMeasureMemberFunc (src/common/Utils.h:17-35): "<label> took <ms>ms".
template <class F>
auto timed(std::ostream& out, const char* label, F&& f) {
    const auto t0 = std::chrono::steady_clock::now();
    auto r = f();
    out << label << " took "
        << std::chrono::duration_cast<std::chrono::milliseconds>(std::chrono::steady_clock::now() - t0).count()
        << "ms\n";
    return r;
}

template <class P>
std::vector<Connection> filter_connections(const std::vector<Connection>& v, P&& p) {   // :126-130
    std::vector<Connection> r;
    std::copy_if(v.begin(), v.end(), std::back_inserter(r), p);
    return r;
}

// get_vectors_intersection (src/common/Utils.h:124-141): sorted inputs, duplicates pairwise.
size_t intersection_size(const std::vector<KmerID>& x, const std::vector<KmerID>& y,
                         std::vector<KmerID>* out = nullptr) {
    size_t i = 0, j = 0, n = 0;
    while (i < x.size() && j < y.size()) {
        if (x[i] < y[j]) {
            ++i;
        } else if (y[j] < x[i]) {
            ++j;
        } else {
            if (out) out->push_back(x[i]);
            ++n;
            ++i;
            ++j;
        }
    }
    return n;
}

std::vector<ComponentList> extract_components(const std::vector<std::pair<ComponentList, SpanningTree>>& v) {
    std::vector<ComponentList> r;   // :700-706
    for (auto& p : v) r.push_back(p.first);
    return r;
}

}  // namespace

// ------------------------------------------------------------------------ union_find (:424-489)
std::vector<std::pair<ComponentList, SpanningTree>> union_find(const std::vector<Connection>& connections,
                                                               const std::set<ComponentID>& restricted,
                                                               int min_component_size, int max_component_size) {
    if (max_component_size == -1) max_component_size = INT_MAX;
    // ids are read ids from one dense range: the same statements over flat arrays indexed by id - lo
    // (hash maps cost ~90 ns an edge on C3's 2 M scaffold-forming connections); the result is in
    // ascending root id, the std::map order of the general version below
    ComponentID lo = UINT32_MAX, hi = 0;
    for (const Connection& c : connections) {
        lo = std::min({lo, c.x, c.y});
        hi = std::max({hi, c.x, c.y});
    }
    if (!connections.empty() && (uint64_t)hi - lo < (1ull << 26)) {
        const size_t N = (size_t)(hi - lo) + 1;
        std::vector<ComponentID> parent(N, UINT32_MAX);   // UINT32_MAX: not a vertex
        std::vector<ComponentList> comp(N);
        std::vector<SpanningTree> tree(N);
        std::vector<uint8_t> restr(N, 0);
        for (const Connection& c : connections)
            for (ComponentID v : {c.x, c.y})
                if (parent[v - lo] == UINT32_MAX) {
                    parent[v - lo] = v;
                    comp[v - lo] = {v};
                    restr[v - lo] = restricted.count(v) != 0;
                }
        auto root = [&](ComponentID v) {
            ComponentID r = v;
            while (parent[r - lo] != r) r = parent[r - lo];
            while (parent[v - lo] != r) {
                const ComponentID n = parent[v - lo];
                parent[v - lo] = r;
                v = n;
            }
            return r;
        };
        for (const Connection& c : connections) {
            const ComponentID px = root(c.x), py = root(c.y);
            if (px == py) continue;
            if (restr[px - lo] && restr[py - lo]) continue;
            if (comp[px - lo].size() + comp[py - lo].size() > (size_t)max_component_size) continue;
            const bool xb = comp[px - lo].size() > comp[py - lo].size();
            const ComponentID bigger = xb ? px : py, smaller = xb ? py : px;
            auto& cb = comp[bigger - lo];
            auto& cs = comp[smaller - lo];
            for (ComponentID id : cs) parent[id - lo] = bigger;
            cb.insert(cb.end(), cs.begin(), cs.end());
            ComponentList().swap(cs);
            auto& tb = tree[bigger - lo];
            tb.emplace_back(c.x, c.y);
            auto& ts = tree[smaller - lo];
            tb.insert(tb.end(), ts.begin(), ts.end());
            SpanningTree().swap(ts);
            restr[bigger - lo] = restr[bigger - lo] || restr[smaller - lo];
        }
        std::vector<std::pair<ComponentList, SpanningTree>> result;
        for (size_t i = 0; i < N; ++i)
            if (parent[i] == lo + (ComponentID)i && comp[i].size() >= (size_t)(int64_t)min_component_size)
                result.emplace_back(std::move(comp[i]), std::move(tree[i]));
        return result;
    }
    std::unordered_map<ComponentID, ComponentID> parents;
    std::map<ComponentID, ComponentList> components;
    std::unordered_map<ComponentID, SpanningTree> trees;
    std::unordered_map<ComponentID, bool> contains_restricted;
    for (const Connection& c : connections)
        for (ComponentID v : {c.x, c.y})
            if (parents.emplace(v, v).second) {
                components[v] = {v};
                trees[v] = {};
                contains_restricted[v] = restricted.count(v) != 0;
            }
    auto get_parent = [&](ComponentID v) {   // with path compression, iteratively
        ComponentID r = v;
        while (parents[r] != r) r = parents[r];
        while (parents[v] != r) {
            const ComponentID n = parents[v];
            parents[v] = r;
            v = n;
        }
        return r;
    };
    for (const Connection& c : connections) {
        const ComponentID px = get_parent(c.x), py = get_parent(c.y);
        if (px == py) continue;
        if (contains_restricted[px] && contains_restricted[py]) continue;
        if (components[px].size() + components[py].size() > (size_t)max_component_size) continue;
        ComponentID bigger, smaller;
        if (components[px].size() > components[py].size()) {
            bigger = px;
            smaller = py;
        } else {
            bigger = py;
            smaller = px;
        }
        for (ComponentID id : components[smaller]) parents[id] = bigger;
        auto& cb = components[bigger];
        auto& cs = components[smaller];
        cb.insert(cb.end(), cs.begin(), cs.end());
        components.erase(smaller);
        auto& tb = trees[bigger];
        tb.emplace_back(c.x, c.y);
        auto& ts = trees[smaller];
        tb.insert(tb.end(), ts.begin(), ts.end());
        trees.erase(smaller);
        contains_restricted[bigger] = contains_restricted[bigger] || contains_restricted[smaller];
        contains_restricted.erase(smaller);
    }
    std::vector<std::pair<ComponentList, SpanningTree>> result;
    for (auto& comp : components)
        if (comp.second.size() >= (size_t)(int64_t)min_component_size)   // int -> size_t as there
            result.emplace_back(comp.second, trees[comp.first]);
    return result;
}

// ------------------------------------------------------------------------ spectral clustering
void sym_eigen(std::vector<double> a, int n, std::vector<double>& values, std::vector<double>& vectors) {
    vectors.assign((size_t)n * n, 0.0);
    for (int i = 0; i < n; ++i) vectors[(size_t)i * n + i] = 1.0;
    auto A = [&](int i, int j) -> double& { return a[(size_t)i * n + j]; };
    auto V = [&](int i, int j) -> double& { return vectors[(size_t)i * n + j]; };
    for (int sweep = 0; sweep < 100; ++sweep) {
        double off = 0.0, diag = 0.0;
        for (int i = 0; i < n; ++i)
            for (int j = 0; j < n; ++j) (i == j ? diag : off) += A(i, j) * A(i, j);
        if (!(off > 1e-30 * std::max(diag, 1e-300))) break;
        for (int p = 0; p < n - 1; ++p)
            for (int q = p + 1; q < n; ++q) {
                const double apq = A(p, q);
                if (apq == 0.0) continue;
                const double theta = (A(q, q) - A(p, p)) / (2.0 * apq);
                const double t = (theta >= 0 ? 1.0 : -1.0) / (std::fabs(theta) + std::sqrt(theta * theta + 1.0));
                const double c = 1.0 / std::sqrt(t * t + 1.0), s = t * c;
                for (int k = 0; k < n; ++k) {   // A <- J^T A J
                    const double akp = A(k, p), akq = A(k, q);
                    A(k, p) = c * akp - s * akq;
                    A(k, q) = s * akp + c * akq;
                }
                for (int k = 0; k < n; ++k) {
                    const double apk = A(p, k), aqk = A(q, k);
                    A(p, k) = c * apk - s * aqk;
                    A(q, k) = s * apk + c * aqk;
                }
                for (int k = 0; k < n; ++k) {
                    const double vkp = V(k, p), vkq = V(k, q);
                    V(k, p) = c * vkp - s * vkq;
                    V(k, q) = s * vkp + c * vkq;
                }
            }
    }
    // ascending eigenvalues (SelfAdjointEigenSolver order), columns permuted alongside
    std::vector<int> ord(n);
    for (int i = 0; i < n; ++i) ord[i] = i;
    std::stable_sort(ord.begin(), ord.end(), [&](int x, int y) { return A(x, x) < A(y, y); });
    values.resize(n);
    std::vector<double> vs((size_t)n * n);
    for (int c = 0; c < n; ++c) {
        values[c] = A(ord[c], ord[c]);
        // sign convention (free in any eigensolver): the largest-magnitude entry is positive
        int big = 0;
        for (int r = 1; r < n; ++r)
            if (std::fabs(V(r, ord[c])) > std::fabs(V(big, ord[c]))) big = r;
        const double sg = V(big, ord[c]) < 0 ? -1.0 : 1.0;
        for (int r = 0; r < n; ++r) vs[(size_t)r * n + c] = sg * V(r, ord[c]);
    }
    vectors.swap(vs);
}

namespace {

// Dense row-major matrix, just enough for Evrot.
struct Mat {
    int r = 0, c = 0;
    std::vector<double> v;
    Mat() = default;
    Mat(int rr, int cc) : r(rr), c(cc), v((size_t)rr * cc, 0.0) {}
    double& operator()(int i, int j) { return v[(size_t)i * c + j]; }
    double operator()(int i, int j) const { return v[(size_t)i * c + j]; }
    static Mat eye(int n) {
        Mat m(n, n);
        for (int i = 0; i < n; ++i) m(i, i) = 1.0;
        return m;
    }
};
Mat mul(const Mat& a, const Mat& b) {
    Mat m(a.r, b.c);
    for (int i = 0; i < a.r; ++i)
        for (int k = 0; k < a.c; ++k) {
            const double x = a(i, k);
            for (int j = 0; j < b.c; ++j) m(i, j) += x * b(k, j);
        }
    return m;
}

// Evrot (src/lib/clustering/Evrot.cpp), method 1 (gradient descent on the Givens angles).
class Evrot {
   public:
    explicit Evrot(const Mat& X) : X_(X), D_(X.c), N_(X.r), A_(D_ * (D_ - 1) / 2), clusters_(D_) {
        for (int i = 0; i < D_ - 1; ++i)   // :22-30
            for (int j = i + 1; j <= D_ - 1; ++j) {
                ik_.push_back(i);
                jk_.push_back(j);
            }
        run();
    }
    double quality() const { return Q_; }
    const std::vector<std::vector<int>>& clusters() const { return clusters_; }
    const Mat& rotated() const { return Xrot_; }

   private:
    void run() {   // :39-123
        const int max_iter = 200;
        std::vector<double> theta(A_, 0.0), theta_new(A_, 0.0);
        double Q = evqual(X_), Q_old1 = Q, Q_old2 = Q;
        int iter = 0;
        while (iter < max_iter) {
            ++iter;
            for (int d = 0; d < A_; ++d) {
                const double alpha = 1.0;
                const double dQ = evqualitygrad(theta, d);
                theta_new[d] = theta[d] - alpha * dQ;
                const double Q_new = evqual(rotate_givens(theta_new));
                if (Q_new > Q) {
                    theta[d] = theta_new[d];
                    Q = Q_new;
                } else {
                    theta_new[d] = theta[d];
                }
            }
            if (iter > 2 && Q - Q_old2 < 1e-3) break;
            Q_old2 = Q_old1;
            Q_old1 = Q;
        }
        Xrot_ = rotate_givens(theta_new);
        cluster_assign();
        Q_ = Q;
    }
    static int argmax_abs(const Mat& m, int i) {   // maxCoeff: first maximum
        int best = 0;
        double bv = std::fabs(m(i, 0));
        for (int j = 1; j < m.c; ++j)
            if (std::fabs(m(i, j)) > bv) {
                bv = std::fabs(m(i, j));
                best = j;
            }
        return best;
    }
    void cluster_assign() {   // :125-143
        std::vector<int> col(N_);
        for (int i = 0; i < N_; ++i) col[i] = argmax_abs(Xrot_, i);
        for (int j = 0; j < D_; ++j)
            for (int i = 0; i < N_; ++i)
                if (col[i] == j) clusters_[j].push_back(i);
    }
    double evqual(const Mat& X) const {   // :145-159
        double sum = 0.0;
        for (int i = 0; i < N_; ++i) {
            double mx = -std::numeric_limits<double>::infinity();
            for (int j = 0; j < D_; ++j) mx = std::max(mx, X(i, j) * X(i, j));
            for (int j = 0; j < D_; ++j) sum += X(i, j) * X(i, j) / mx;
        }
        return 1.0 - (sum / N_ - 1.0) / D_;
    }
    double evqualitygrad(const std::vector<double>& theta, int k) const {   // :161-203
        Mat V(D_, D_);
        V(ik_[k], ik_[k]) = -std::sin(theta[k]);
        V(ik_[k], jk_[k]) = std::cos(theta[k]);
        V(jk_[k], ik_[k]) = -std::cos(theta[k]);
        V(jk_[k], jk_[k]) = -std::sin(theta[k]);
        const Mat U1 = build_Uab(theta, 0, k - 1), U2 = build_Uab(theta, k + 1, A_ - 1);
        const Mat A = mul(mul(mul(X_, U1), V), U2);
        const Mat Y = rotate_givens(theta);
        std::vector<double> mv(N_);
        std::vector<int> mc(N_);
        for (int i = 0; i < N_; ++i) {
            mc[i] = argmax_abs(Y, i);
            mv[i] = Y(i, mc[i]);
        }
        double dJ = 0.0;
        for (int j = 0; j < D_; ++j)
            for (int i = 0; i < N_; ++i) {
                const double t1 = A(i, j) * Y(i, j) / (mv[i] * mv[i]);
                const double t2 = A(i, mc[i]) * (Y(i, j) * Y(i, j)) / (mv[i] * mv[i] * mv[i]);
                dJ += t1 - t2;
            }
        return 2 * dJ / N_ / D_;
    }
    Mat rotate_givens(const std::vector<double>& theta) const { return mul(X_, build_Uab(theta, 0, A_ - 1)); }
    Mat build_Uab(const std::vector<double>& theta, int a, int b) const {   // :213-234
        Mat U = Mat::eye(D_);
        if (b < a) return U;
        for (int k = a; k <= b; ++k) {
            const double tt = theta[k];
            for (int i = 0; i < D_; ++i) {
                const double u_ik = U(i, ik_[k]) * std::cos(tt) - U(i, jk_[k]) * std::sin(tt);
                U(i, jk_[k]) = U(i, ik_[k]) * std::sin(tt) + U(i, jk_[k]) * std::cos(tt);
                U(i, ik_[k]) = u_ik;
            }
        }
        return U;
    }

    Mat X_;
    int D_, N_, A_;
    std::vector<int> ik_, jk_;
    Mat Xrot_;
    double Q_ = 0.0;
    std::vector<std::vector<int>> clusters_;
};

// ClusterRotate::cluster (src/lib/clustering/ClusterRotate.cpp:20-76).
std::vector<std::vector<int>> cluster_rotate(const Mat& X) {
    double max_quality = 0.0;
    std::vector<std::vector<int>> clusters;
    Mat vec_rot;
    Mat vec_in(X.r, 2);
    for (int i = 0; i < X.r; ++i)
        for (int j = 0; j < 2; ++j) vec_in(i, j) = X(i, j);
    std::unique_ptr<Evrot> e;
    for (int g = 2; g <= X.c; ++g) {
        if (g > 2) {
            const Mat prev = e->rotated();
            vec_in = Mat(X.r, g);
            for (int i = 0; i < X.r; ++i) {
                for (int j = 0; j < g - 1; ++j) vec_in(i, j) = prev(i, j);
                vec_in(i, g - 1) = X(i, g - 1);
            }
        }
        e = std::make_unique<Evrot>(vec_in);
        if (e->quality() > max_quality) max_quality = e->quality();
        if (e->quality() > max_quality || max_quality - e->quality() <= 0.001) {
            clusters = e->clusters();
            vec_rot = e->rotated();
        }
    }
    Mat centres((int)clusters.size(), vec_rot.c);
    for (size_t i = 0; i < clusters.size(); ++i) {
        for (int p : clusters[i])
            for (int j = 0; j < vec_rot.c; ++j) centres((int)i, j) += vec_rot(p, j);
        for (int j = 0; j < vec_rot.c; ++j) centres((int)i, j) /= (double)clusters[i].size();
    }
    for (size_t i = 0; i < clusters.size(); ++i) {   // ascending distance to the centre (multimap)
        std::vector<std::pair<double, int>> d;
        for (int p : clusters[i]) {
            double d2 = 0.0;
            for (int j = 0; j < vec_rot.c; ++j) d2 += (vec_rot(p, j) - centres((int)i, j)) * (vec_rot(p, j) - centres((int)i, j));
            d.emplace_back(d2, p);
        }
        std::stable_sort(d.begin(), d.end(), [](auto& a, auto& b) { return a.first < b.first; });
        clusters[i].clear();
        for (auto& x : d) clusters[i].push_back(x.second);
    }
    return clusters;
}

}  // namespace

std::vector<ComponentList> spectral_clustering(const std::vector<Connection>& connections, int dims) {
    // :653-697
    std::unordered_map<ComponentID, int> to_id;
    std::vector<ComponentID> id_to;
    std::vector<Score> scores;
    for (const Connection& c : connections) {
        for (ComponentID v : {c.x, c.y})
            if (to_id.emplace(v, (int)id_to.size()).second) id_to.push_back(v);
        scores.push_back(c.score);
    }
    if (scores.empty()) return {};
    const int max_exponent = 20;
    const int n = (int)id_to.size();
    if (n > 8192) throw std::runtime_error("spectral clustering of " + std::to_string(n) +
                                           " components exceeds the dense affinity-matrix limit (8192)");
    std::vector<double> m((size_t)n * n, 0.0);
    const Score max_score = *std::max_element(scores.begin(), scores.end());
    const Score min_score = *std::min_element(scores.begin(), scores.end());
    // Every score equal (e.g. one strong connection): scale_strength is 0/0 = NaN for every edge there
    // (:672-674) and the whole affinity matrix NaN; Eigen2's eigenvectors of it are unspecified (parity
    // unpinned).  Here that case is explicit: no grouping, every component its own cluster (what the NaN
    // matrix gave through this eigensolver and rotation), so merge_components changes nothing.
    if (max_score == min_score) {
        std::vector<ComponentList> alone;
        for (ComponentID v : id_to) alone.push_back({v});
        return alone;
    }
    auto scale = [&](Score s) {
        return ((double)(max_exponent - 0.3) * (double)(s - min_score)) / (double)(max_score - min_score) + 0.3;
    };
    for (const Connection& c : connections) {
        const int x = to_id[c.x], y = to_id[c.y];
        const double w = std::exp(scale(c.score));
        m[(size_t)x * n + y] = w;
        m[(size_t)y * n + x] = w;
    }
    dims = std::min(n, dims);
    // SpectralClustering (src/lib/clustering/SpectralClustering.cpp:20-53): normalised
    // Laplacian Deg^-1/2 m Deg^-1/2, eigenvectors ordered by descending eigenvalue
    std::vector<double> deg(n);
    for (int i = 0; i < n; ++i) {
        double s = 0.0;
        for (int j = 0; j < n; ++j) s += m[(size_t)i * n + j];
        deg[i] = 1 / std::sqrt(s);
    }
    std::vector<double> lap((size_t)n * n);
    for (int i = 0; i < n; ++i)
        for (int j = 0; j < n; ++j) lap[(size_t)i * n + j] = deg[i] * m[(size_t)i * n + j] * deg[j];
    std::vector<double> val, vec;
    sym_eigen(lap, n, val, vec);
    for (int i = 0; i < n - 1; ++i) {   // selection sort, largest first (:37-45)
        int k = 0;
        double best = val[i];
        for (int t = 1; t < n - i; ++t)
            if (val[i + t] > best) {
                best = val[i + t];
                k = t;
            }
        if (k > 0) {
            std::swap(val[i], val[k + i]);
            for (int r = 0; r < n; ++r) std::swap(vec[(size_t)r * n + i], vec[(size_t)r * n + k + i]);
        }
    }
    Mat X(n, dims);
    for (int r = 0; r < n; ++r)
        for (int c = 0; c < dims; ++c) X(r, c) = vec[(size_t)r * n + c];
    if (dims < 2) {   // ClusterRotate needs two columns; one component per cluster
        std::vector<ComponentList> one{ComponentList(id_to.begin(), id_to.end())};
        return one;
    }
    const auto clusters = cluster_rotate(X);
    std::vector<ComponentList> result(clusters.size());
    for (size_t i = 0; i < clusters.size(); ++i)
        for (int id : clusters[i]) result[i].push_back(id_to[id]);
    return result;
}

// ------------------------------------------------------------------------ engine
ClusteringEngine::ClusteringEngine(const ClusteringConfig& cfg, bool debug, const RecordSet& reads,
                                   uint32_t first_read_id, std::vector<uint64_t> hit_ptr,
                                   std::vector<uint32_t> sorted_kid, std::vector<uint64_t> first_ptr,
                                   std::vector<uint32_t> first_kid, std::vector<uint32_t> first_pos,
                                   const std::vector<uint64_t>& kci_ptr, const std::vector<uint32_t>& kci_read,
                                   hga_ctx* gpu)
    : cfg_(cfg),
      debug_(debug),
      reads_(reads),
      first_id_(first_read_id),
      hit_ptr_(std::move(hit_ptr)),
      first_ptr_(std::move(first_ptr)),
      first_kid_(std::move(first_kid)),
      first_pos_(std::move(first_pos)),
      gpu_(gpu) {
    const uint64_t n = reads.size();
    if (hit_ptr_.size() != n + 1 || first_ptr_.size() != n + 1)
        throw std::invalid_argument("index arrays do not match the reads");
    for (uint64_t i = 0; i < n; ++i) {   // construct_indices :256-276
        if (hit_ptr_[i + 1] == hit_ptr_[i]) continue;
        Component c;
        c.reads = {first_id_ + (uint32_t)i};
        c.kmers.assign(sorted_kid.begin() + (int64_t)hit_ptr_[i], sorted_kid.begin() + (int64_t)hit_ptr_[i + 1]);
        c.categories = {reads.category[i]};
        index_.emplace_hint(index_.end(), first_id_ + (uint32_t)i, std::move(c));
    }
    // (built serially: the same construction on the host threads measured slower, 100 -> 155 ms at C3 —
    // 1.9 M small allocations contend in the allocator)
    kci_.resize(kci_ptr.empty() ? 0 : kci_ptr.size() - 1);
    for (size_t k = 0; k + 1 < kci_ptr.size(); ++k)
        kci_[k].assign(kci_read.begin() + (int64_t)kci_ptr[k], kci_read.begin() + (int64_t)kci_ptr[k + 1]);
}

uint32_t ClusteringEngine::read_length(ComponentID r) const {   // ReadMetaData::length
    const uint64_t i = r - first_id_;
    return (uint32_t)(reads_.offsets[i + 1] - reads_.offsets[i]);
}

// read_metas[x].kmer_positions[kmer_id]: first occurrence, 0 (operator[] default) when absent.
uint32_t ClusteringEngine::kmer_position(ComponentID r, KmerID kid) const {
    const uint64_t i = r - first_id_;
    const auto b = first_kid_.begin() + (int64_t)first_ptr_[i], e = first_kid_.begin() + (int64_t)first_ptr_[i + 1];
    const auto it = std::lower_bound(b, e, kid);
    return it != e && *it == kid ? first_pos_[(size_t)(it - first_kid_.begin())] : 0u;
}

bool ClusteringEngine::is_good(ComponentID x, ComponentID y) const {
    if (!debug_) return false;
    const auto a = index_.find(x), b = index_.find(y);
    return a != index_.end() && b != index_.end() && a->second.categories == b->second.categories;
}

// get_connections (:301-333) on the host state.
std::vector<Connection> ClusteringEngine::host_connections(const std::vector<ComponentID>& pivots,
                                                           Score min_score) const {
    const ComponentID max_id = first_id_ + (ComponentID)reads_.size();
    const int T = std::max(1, std::min<int>(host_threads(), (int)pivots.size()));
    std::vector<std::vector<Connection>> part(T);
    std::atomic<size_t> next{0};
    auto work = [&](int t) {
        std::vector<Score> cnt(max_id + 1, 0);
        std::vector<ComponentID> touched;
        size_t q;
        while ((q = next.fetch_add(1)) < pivots.size()) {
            const ComponentID p = pivots[q];
            const auto it = index_.find(p);
            if (it == index_.end()) continue;
            for (KmerID kid : it->second.kmers)
                for (ComponentID c : kci_[kid])
                    if (cnt[c]++ == 0) touched.push_back(c);
            for (ComponentID c : touched) {
                if (c != p && cnt[c] >= min_score) part[t].push_back({p, c, cnt[c], is_good(p, c)});
                cnt[c] = 0;
            }
            touched.clear();
        }
    };
    std::vector<std::thread> th;
    for (int t = 1; t < T; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    std::vector<Connection> out;
    for (auto& p : part) out.insert(out.end(), p.begin(), p.end());
    sort_connections(out);
    return out;
}

std::vector<Connection> ClusteringEngine::get_connections(const std::vector<ComponentID>& pivots, Score min_score,
                                                          uint32_t min_kmers, double keep_fraction) {
    const auto prefix = [keep_fraction](std::vector<Connection> v) {
        if (keep_fraction >= 0) v.resize(std::min(v.size(), (size_t)((double)v.size() * keep_fraction)));
        return v;
    };
    if (!(pristine_ && (gpu_ || dev_conn_))) return prefix(host_connections(pivots, min_score));
    if (min_kmers == 0 && pivots.empty()) return {};   // (a null pivot list means "every read" there)
    if (dev_conn_) {
        ++gpu_calls_;
        return prefix(dev_conn_(pivots, min_score, min_kmers));
    }
    // construct_indices' state is on the device: hga_connections_run (connect.hip)
    std::vector<int32_t> cats;
    if (debug_) cats.assign(reads_.category.begin(), reads_.category.end());
    uint64_t n = 0;
    const bool all = min_kmers > 0;   // every component with >= min_kmers KmerIDs (filter_components)
    if (hga_connections_run(gpu_, all ? nullptr : pivots.data(), all ? 0 : pivots.size(), all ? min_kmers : 1,
                            min_score, debug_ ? cats.data() : nullptr, &n) != HGA_OK)
        throw std::runtime_error(std::string("hga_connections_run: ") + hga_last_error());
    if (keep_fraction >= 0) n = std::min<uint64_t>(n, (uint64_t)(size_t)((double)n * keep_fraction));
    std::vector<uint32_t> x(n), y(n);
    std::vector<uint64_t> s(n);
    std::vector<uint8_t> g(n);
    if (hga_connections_fetch_range(gpu_, 0, n, x.data(), y.data(), s.data(), g.data()) != HGA_OK)
        throw std::runtime_error(std::string("hga_connections_fetch_range: ") + hga_last_error());
    ++gpu_calls_;
    std::vector<Connection> out(n);
    for (uint64_t i = 0; i < n; ++i) out[i] = {x[i], y[i], s[i], g[i] != 0};
    return out;
}

std::vector<Connection> ClusteringEngine::get_all_connections(Score min_score, double keep_fraction) {   // :335-339
    if (pristine_ && (gpu_ || dev_conn_)) return get_connections({}, min_score, 1, keep_fraction);
    std::vector<ComponentID> ids;
    for (auto& kv : index_) ids.push_back(kv.first);
    return get_connections(ids, min_score, 0, keep_fraction);
}

// accumulate_kmer_ids (:341-347): merge_n_vectors(..., unique = true), a sorted set union.
std::vector<KmerID> ClusteringEngine::accumulate_kmer_ids(const std::vector<ComponentID>& ids) const {
    std::vector<KmerID> all;
    for (ComponentID id : ids) {
        const auto it = index_.find(id);
        if (it != index_.end()) all.insert(all.end(), it->second.kmers.begin(), it->second.kmers.end());
    }
    std::sort(all.begin(), all.end());
    all.erase(std::unique(all.begin(), all.end()), all.end());
    return all;
}

// merge_components (:349-422).  Same statements, flat data structures: a survivor's KmerID union
// is a mark pass over the dense KmerID range when the members hold many ids (a sort of the
// concatenation otherwise), and the removal lists are a counting sort of (KmerID, component) pairs
// by KmerID instead of an ordered map of vectors — on C3, where one component absorbs most reads
// (~20 M pairs), the map took 17.8 s.  The kmer_component_index update runs over the host threads.
std::vector<ComponentID> ClusteringEngine::merge_components(const std::vector<ComponentList>& components) {
    using clk = std::chrono::steady_clock;
    const auto t_start = clk::now();
    std::vector<ComponentID> merged_ids;
    const size_t nk = kci_.size();
    const int HT = std::max(1, host_threads());
    // ranges [0, n) split over up to HT threads (the calling thread takes the last one)
    auto par = [&](size_t n, size_t grain, const std::function<void(int, size_t, size_t)>& f) {
        const int T = (int)std::max<size_t>(1, std::min<size_t>((size_t)HT, n / std::max<size_t>(grain, 1)));
        std::vector<std::thread> th;
        for (int t = 0; t < T; ++t) {
            const size_t a = n * (size_t)t / (size_t)T, b = n * (size_t)(t + 1) / (size_t)T;
            if (t + 1 == T) f(t, a, b);
            else th.emplace_back(f, t, a, b);
        }
        for (auto& x : th) x.join();
        return T;
    };
    // (KmerID << 32 | component) pairs, per thread; their order is irrelevant: each KmerID's removal
    // list is sorted before use
    std::vector<std::vector<uint64_t>> pairs((size_t)HT);
    std::vector<uint8_t> mark;
    double t_members = 0, t_union = 0, t_pairs = 0;   // (HGA_TIMING parts of merge.groups)
    for (const ComponentList& ids : components) {
        if (ids.empty()) continue;   // (an empty spectral cluster would dereference ids[0] there)
        if (ids.size() == 1) {
            merged_ids.push_back(ids[0]);
            continue;
        }
        const auto q0 = clk::now();
        std::set<int32_t> cats;
        std::vector<uint32_t> contained;
        size_t total = 0;
        std::vector<const std::vector<KmerID>*> km(ids.size());
        for (size_t i = 0; i < ids.size(); ++i) {
            Component& c = index_.at(ids[i]);
            contained.insert(contained.end(), c.reads.begin(), c.reads.end());
            c.reads.clear();
            cats.insert(c.categories.begin(), c.categories.end());
            total += c.kmers.size();
            km[i] = &c.kmers;
        }
        const auto q1 = clk::now();
        std::vector<KmerID> acc;
        if (total > nk / 16 + 64) {   // accumulate_kmer_ids as a mark pass (ids < nk), both halves threaded
            if (mark.empty()) mark.assign(nk, 0);
            par(ids.size(), 64, [&](int, size_t a, size_t b) {
                for (size_t i = a; i < b; ++i)
                    for (KmerID kid : *km[i]) std::atomic_ref<uint8_t>(mark[kid]).store(1, std::memory_order_relaxed);
            });
            std::vector<std::vector<KmerID>> part((size_t)HT);
            const int T = par(nk, 1 << 16, [&](int t, size_t a, size_t b) {
                for (size_t kid = a; kid < b; ++kid)
                    if (mark[kid]) {
                        part[(size_t)t].push_back((KmerID)kid);
                        mark[kid] = 0;
                    }
            });
            for (int t = 0; t < T; ++t) acc.insert(acc.end(), part[(size_t)t].begin(), part[(size_t)t].end());
        } else {
            acc = accumulate_kmer_ids(ids);
        }
        Component& survivor = index_.at(ids[0]);
        survivor.kmers = std::move(acc);
        survivor.categories = cats;
        survivor.reads = contained;
        merged_ids.push_back(ids[0]);
        km[0] = &survivor.kmers;
        const auto q2 = clk::now();
        par(ids.size(), 64, [&](int t, size_t a, size_t b) {
            auto& pv = pairs[(size_t)t];
            size_t add = 0;
            for (size_t i = a; i < b; ++i) add += km[i]->size();
            if (pv.capacity() < pv.size() + add) pv.reserve(std::max(pv.size() + add, 2 * pv.capacity()));
            for (size_t i = a; i < b; ++i)
                for (KmerID kid : *km[i]) pv.push_back((uint64_t)kid << 32 | ids[i]);
        });
        pristine_ = false;
        const auto q3 = clk::now();
        t_members += std::chrono::duration<double, std::milli>(q1 - q0).count();
        t_union += std::chrono::duration<double, std::milli>(q2 - q1).count();
        t_pairs += std::chrono::duration<double, std::milli>(q3 - q2).count();
    }
    size_t npairs = 0;
    for (auto& pv : pairs) npairs += pv.size();
    if (npairs == 0) return merged_ids;
    const auto t_groups = clk::now();
    // removal lists: a counting sort of the pairs by KmerID over the threads without atomics — a count
    // row per pair vector, per-KmerID totals and their prefix, then each vector's cursors per KmerID
    // (its rows become cursors) and its own scatter
    const size_t nv = pairs.size();
    if (npairs >= UINT32_MAX) {   // (u32 cursors) one vector of everything, counted serially
        for (size_t v = 1; v < nv; ++v) {
            pairs[0].insert(pairs[0].end(), pairs[v].begin(), pairs[v].end());
            std::vector<uint64_t>().swap(pairs[v]);
        }
    }
    std::vector<std::vector<uint32_t>> cnt(nv);
    par(nv, 1, [&](int, size_t a, size_t b) {
        for (size_t v = a; v < b; ++v) {
            if (pairs[v].empty()) continue;
            cnt[v].assign(nk, 0);
            for (uint64_t pr : pairs[v]) ++cnt[v][pr >> 32];
        }
    });
    std::vector<uint64_t> start(nk + 1, 0);
    par(nk, 1 << 14, [&](int, size_t a, size_t b) {
        for (size_t k = a; k < b; ++k) {
            uint64_t t = 0;
            for (size_t v = 0; v < nv; ++v)
                if (!cnt[v].empty()) t += cnt[v][k];
            start[k + 1] = t;
        }
    });
    for (size_t k = 0; k < nk; ++k) start[k + 1] += start[k];
    if (npairs < UINT32_MAX) par(nk, 1 << 14, [&](int, size_t a, size_t b) {   // counts -> each vector's first slot per KmerID
        for (size_t k = a; k < b; ++k) {
            uint64_t o = start[k];
            for (size_t v = 0; v < nv; ++v)
                if (!cnt[v].empty()) {
                    const uint32_t c = cnt[v][k];
                    cnt[v][k] = (uint32_t)o;
                    o += c;
                }
        }
    });
    std::vector<ComponentID> rem(npairs);
    if (npairs >= UINT32_MAX) {
        std::vector<uint64_t> cur(start.begin(), start.end() - 1);
        for (uint64_t pr : pairs[0]) rem[cur[pr >> 32]++] = (ComponentID)pr;
    } else {
        par(nv, 1, [&](int, size_t a, size_t b) {
            for (size_t v = a; v < b; ++v)
                for (uint64_t pr : pairs[v]) rem[cnt[v][pr >> 32]++] = (ComponentID)pr;
        });
    }
    pairs.clear();
    pairs.shrink_to_fit();
    // kmer_component_index update (:395-419), including its early stop: once the removal list
    // is exhausted the rest of the kmer's list is not copied
    auto update = [&](size_t k0, size_t k1) {
        for (size_t kid = k0; kid < k1; ++kid) {
            if (start[kid] == start[kid + 1]) continue;
            ComponentID* rb = rem.data() + start[kid];
            ComponentID* re = rem.data() + start[kid + 1];
            // (the scatter keeps each pair vector's member order, so with ascending member lists the
            // removal list usually arrives sorted)
            if (!std::is_sorted(rb, re)) std::sort(rb, re);
            std::vector<ComponentID>& list = kci_[kid];
            size_t j = 0, w = 0;   // kept entries compacted in place (w <= j): the reference's `updated`
            for (ComponentID* r = rb; r < re && j < list.size();) {
                if (*r < list[j]) {
                    ++r;
                } else if (list[j] < *r) {
                    list[w++] = list[j++];
                } else {
                    ++r;
                    ++j;
                }
            }
            list.resize(w);
        }
    };
    const int T = std::max(1, std::min<int>(host_threads(), (int)(rem.size() >> 16) + 1));
    std::vector<std::thread> th;
    size_t k0 = 0;
    for (int t = 0; t < T; ++t) {   // kid ranges of about equal pair counts
        const uint64_t want = (uint64_t)rem.size() * (uint64_t)(t + 1) / (uint64_t)T;
        const size_t k1 = t + 1 == T ? nk : (size_t)(std::upper_bound(start.begin(), start.end(), want) - start.begin()) - 1;
        const size_t e = std::max(k0, std::min(k1, nk));
        if (t + 1 == T) update(k0, nk);
        else th.emplace_back(update, k0, e);
        k0 = e;
    }
    for (auto& x : th) x.join();
    if (const char* te = std::getenv("HGA_TIMING"); te && std::string(te) == "1") {
        auto ms = [](clk::time_point a, clk::time_point b) { return std::chrono::duration<double, std::milli>(b - a).count(); };
        static int call = 0;   // one set of lines per call: merge<call>.*
        ++call;
        std::fprintf(stderr,
                     "hga-timing merge%d.groups %.2f\nhga-timing merge%d.members %.2f\nhga-timing merge%d.union %.2f\n"
                     "hga-timing merge%d.pairs %.2f\nhga-timing merge%d.kci_update %.2f\n",
                     call, ms(t_start, t_groups), call, t_members, call, t_union, call, t_pairs, call,
                     ms(t_groups, clk::now()));
    }
    return merged_ids;
}

void ClusteringEngine::remove_merged_components() {   // :718-725
    for (auto it = index_.begin(); it != index_.end();) {
        if (it->second.reads.empty()) it = index_.erase(it);
        else ++it;
    }
}

std::vector<ComponentID> ClusteringEngine::component_ids(uint64_t threshold_size) const {   // :727-735
    std::vector<ComponentID> r;
    for (auto& kv : index_)
        if (kv.second.reads.size() >= threshold_size) r.push_back(kv.first);
    return r;
}

// approximate_read_overlap (:491-507).
int ClusteringEngine::approximate_read_overlap(ComponentID x, ComponentID y) const {
    std::vector<KmerID> shared;
    intersection_size(index_.at(x).kmers, index_.at(y).kmers, &shared);
    if (shared.empty()) return 0;   // (max_element of an empty range there)
    int max_x = INT_MIN, max_y = INT_MIN, min_x = INT_MAX, min_y = INT_MAX;
    for (KmerID kid : shared) {
        const int px = (int)kmer_position(x, kid), py = (int)kmer_position(y, kid);
        max_x = std::max(max_x, px);
        min_x = std::min(min_x, px);
        max_y = std::max(max_y, py);
        min_y = std::min(min_y, py);
    }
    return std::max(max_x - min_x, max_y - min_y);
}

// get_spanning_tree_tails (:509-573).
std::pair<std::vector<ComponentID>, std::vector<ComponentID>> ClusteringEngine::spanning_tree_tails(
    const SpanningTree& tree) const {
    std::map<ComponentID, std::map<ComponentID, int>> adjacency;
    // the edges' overlaps (an intersection of two merged components' KmerID lists each: the stage's
    // cost) on the host threads, then the adjacency built in tree order as before
    std::vector<int> ov(tree.size());
    {
        const int T = std::max(1, std::min<int>(host_threads(), (int)(tree.size() / 8) + 1));
        std::atomic<size_t> next{0};
        auto work = [&] {
            size_t q;
            while ((q = next.fetch_add(1)) < tree.size()) ov[q] = approximate_read_overlap(tree[q].first, tree[q].second);
        };
        std::vector<std::thread> th;
        for (int t = 1; t < T; ++t) th.emplace_back(work);
        work();
        for (auto& x : th) x.join();
    }
    for (size_t q = 0; q < tree.size(); ++q) {
        const auto& edge = tree[q];
        adjacency[edge.first].emplace(edge.second, ov[q]);
        adjacency[edge.second].emplace(edge.first, ov[q]);
    }
    if (adjacency.empty()) return {};
    auto distance_bfs = [&](ComponentID start) {
        std::queue<ComponentID> q;
        q.push(start);
        std::set<ComponentID> visited;
        std::map<ComponentID, uint64_t> dist{{start, (uint64_t)read_length(start)}};
        while (!q.empty()) {
            const ComponentID v = q.front();
            visited.insert(v);
            q.pop();
            const auto it = adjacency.find(v);
            if (it == adjacency.end()) continue;
            for (auto& a : it->second)
                if (!visited.count(a.first)) {   // unsigned arithmetic as in :529
                    dist[a.first] = dist[v] + read_length(a.first) - (uint64_t)(int64_t)a.second;
                    q.push(a.first);
                }
        }
        return dist;
    };
    auto max_pair = [](const std::map<ComponentID, uint64_t>& d) {
        auto best = d.begin();
        for (auto it = d.begin(); it != d.end(); ++it)
            if (best->second < it->second) best = it;
        return *best;
    };
    const auto initial = distance_bfs(adjacency.begin()->first);
    const auto farthest = max_pair(initial);
    std::vector<ComponentID> left, right;
    const uint64_t tail_length = reads_.meta.avg_read_length * 2;
    const auto to_right = distance_bfs(farthest.first);
    const auto far_right = max_pair(to_right);
    for (auto& vd : to_right)
        if (vd.second + tail_length > far_right.second) right.push_back(vd.first);
    const auto to_left = distance_bfs(far_right.first);
    const auto far_left = max_pair(to_left);
    for (auto& vd : to_left)
        if (vd.second + tail_length > far_left.second) left.push_back(vd.first);
    return {left, right};
}

// amplify_component (:575-584).
std::vector<ComponentID> ClusteringEngine::amplify_component(const std::vector<ComponentID>& comp, Score min_score) {
    const auto conns = get_connections(comp, min_score);
    std::set<ComponentID> ids(comp.begin(), comp.end());
    for (auto& c : conns) {
        ids.insert(c.x);
        ids.insert(c.y);
    }
    return std::vector<ComponentID>(ids.begin(), ids.end());
}

// get_core_component_connections (:586-651).
std::vector<Connection> ClusteringEngine::core_component_connections(
    const std::vector<std::pair<ComponentList, SpanningTree>>& comps_and_trees) {
    std::map<ComponentID, std::pair<std::vector<KmerID>, std::vector<KmerID>>> tails_map;
    // HGA_TIMING=1: the stage's parts summed over the scaffold components ("hga-timing tails.<part> <ms>")
    using clk = std::chrono::steady_clock;
    double t_tree = 0, t_amp = 0, t_acc = 0;
    auto since = [](clk::time_point a) { return std::chrono::duration<double, std::milli>(clk::now() - a).count(); };
    for (auto& ct : comps_and_trees) {
        auto t0 = clk::now();
        const auto tails = spanning_tree_tails(ct.second);
        t_tree += since(t0);
        t0 = clk::now();
        const auto lv = amplify_component(tails.first, (Score)(int)cfg_.tail_amplification_min_score);
        const auto rv = amplify_component(tails.second, (Score)(int)cfg_.tail_amplification_min_score);
        t_amp += since(t0);
        t0 = clk::now();
        tails_map.emplace(ct.first[0], std::make_pair(accumulate_kmer_ids(lv), accumulate_kmer_ids(rv)));
        t_acc += since(t0);
    }
    const auto t_int0 = clk::now();
    std::vector<Connection> edges;
    for (auto& a : tails_map)
        for (auto& b : tails_map)
            if (a.first < b.first) {
                const Score s[4] = {intersection_size(a.second.first, b.second.first),
                                    intersection_size(a.second.first, b.second.second),
                                    intersection_size(a.second.second, b.second.first),
                                    intersection_size(a.second.second, b.second.second)};
                edges.push_back({a.first, b.first, *std::max_element(s, s + 4), is_good(a.first, b.first)});
            }
    sort_connections(edges);
    if (const char* te = std::getenv("HGA_TIMING"); te && std::string(te) == "1")
        std::fprintf(stderr, "hga-timing tails.spanning_tree_tails %.2f\nhga-timing tails.amplify %.2f\n"
                             "hga-timing tails.accumulate %.2f\nhga-timing tails.intersections %.2f\n",
                     t_tree, t_amp, t_acc, since(t_int0));
    return filter_connections(edges, [](const Connection& c) { return c.score > 0; });
}

// ReadComponent::to_string (ReadClusteringEngine.h:98-112) with consistency (:52-64) and
// category_intervals (:66-96): read counts per category, categories 0 and 1 always listed, joined by
// "/"; per category present, the union of the reads' [start, end] simulator coordinates as
// "(a,b)" joined by ";", categories joined by " / ".
std::string ClusteringEngine::component_string(ComponentID id) const {
    const Component& c = index_.at(id);
    std::map<int32_t, int> counts{{0, 0}, {1, 0}};
    std::map<int32_t, std::vector<std::pair<uint32_t, bool>>> endpoints;   // Endpoint = (position, is start)
    for (uint32_t r : c.reads) {
        const uint64_t i = r - first_id_;
        const int32_t cat = reads_.category[i];
        ++counts[cat];
        auto& e = endpoints[cat];
        e.emplace_back(reads_.start.empty() ? 0u : reads_.start[i], true);
        e.emplace_back(reads_.end.empty() ? 0u : reads_.end[i], false);
    }
    std::string s = "#" + std::to_string(id) + " : ";
    bool first = true;
    for (auto& kv : counts) {
        if (!first) s += "/";
        s += std::to_string(kv.second);
        first = false;
    }
    s += " [";
    first = true;
    for (auto& kv : endpoints) {
        auto& e = kv.second;
        std::sort(e.begin(), e.end());   // (position, false) before (position, true), as std::pair orders them
        if (!first) s += " / ";
        first = false;
        uint32_t open_at = 0;   // (uninitialised there until the first opening endpoint)
        int opened = 0;
        bool any = false;
        for (auto& ep : e) {
            if (ep.second) {
                if (++opened == 1) open_at = ep.first;
            } else if (--opened == 0) {
                if (any) s += ";";
                s += "(" + std::to_string(open_at) + "," + std::to_string(ep.first) + ")";
                any = true;
            }
        }
    }
    s += "]";
    return s;
}

void ClusteringEngine::print_components(std::vector<ComponentID>& ids, std::ostream& out) const {
    if (!debug_) return;
    std::stable_sort(ids.begin(), ids.end(), [this](ComponentID x, ComponentID y) {
        const size_t a = index_.at(x).reads.size(), b = index_.at(y).reads.size();
        return a != b ? a > b : x < y;
    });
    out << "### Printing " << ids.size() << " components ###\n";
    for (ComponentID id : ids) out << component_string(id) << "\n";
    out << "### ###\n\n";
    out.flush();
}

// run_clustering after construct_indices (:737-801).
std::vector<ComponentID> ClusteringEngine::run(std::ostream& out) {
    if (cfg_.force_spectral) {   // :739-746
        auto conns = timed(out, "Calculation of connections between reads", [&] { return get_all_connections(5); });
        auto spectral = timed(out, "Forced spectral clustering",
                              [&] { return spectral_clustering(conns, cfg_.spectral_dims); });
        merge_components(spectral);
        auto ids = component_ids((uint64_t)(int64_t)cfg_.scaffold_component_min_size);
        print_components(ids, out);   // :745
        return ids;
    }
    std::vector<Connection> scaffold_forming, conns;
    if (cfg_.scaffold_forming_score > 0) {   // :749-756
        const Score s = cfg_.scaffold_forming_score;
        conns = timed(out, "Calculation of connections between reads", [&] {
            if (pristine_ && gpu_) return get_connections({}, s, (uint32_t)std::min<Score>(s, UINT32_MAX));
            std::vector<ComponentID> ids;
            for (auto& kv : index_)
                if (kv.second.kmers.size() >= s) ids.push_back(kv.first);
            return get_connections(ids, s);
        });
        scaffold_forming = filter_connections(conns, [&](const Connection& c) { return c.score > s; });
    } else {
        // only the first size * fraction entries are used (:754-755): fetch just that prefix
        scaffold_forming = timed(out, "Calculation of connections between reads",
                                 [&] { return get_all_connections(1, cfg_.scaffold_forming_fraction); });
    }
    std::set<ComponentID> restricted;
    auto comps_and_trees = timed(out, "Union-find", [&] {
        return union_find(scaffold_forming, restricted, cfg_.scaffold_component_min_size,
                          cfg_.scaffold_component_max_size);
    });
    auto scaffold_ids = timed(out, "Merging of initial components",
                              [&] { return merge_components(extract_components(comps_and_trees)); });
    print_components(scaffold_ids, out);   // :766
    if (scaffold_ids.size() > 2) {   // :768-777
        auto core = timed(out, "Calculation of tail connections", [&] { return core_component_connections(comps_and_trees); });
        auto strong = filter_connections(core, [](const Connection& c) { return c.score > 5; });
        if (!strong.empty()) {
            auto spectral = timed(out, "Spectral clustering", [&] { return spectral_clustering(strong, cfg_.spectral_dims); });
            timed(out, "Merging of scaffold components", [&] { return merge_components(spectral); });
        }
        remove_merged_components();
    }
    const uint64_t min_size = (uint64_t)(int64_t)cfg_.scaffold_component_min_size;   // int -> u64 as there
    auto core_ids = component_ids(min_size);
    print_components(core_ids, out);   // :781 (sorts core_ids in place, as there)
    {   // :785-794
        conns = timed(out, "Calculation of enrichment connections",
                      [&] { return get_connections(core_ids, cfg_.enrichment_connections_min_score); });
        restricted.insert(core_ids.begin(), core_ids.end());
        comps_and_trees = union_find(conns, restricted, 2, -1);
        timed(out, "Merging into core components", [&] { return merge_components(extract_components(comps_and_trees)); });
        remove_merged_components();
        core_ids = component_ids(min_size);
    }
    print_components(core_ids, out);   // :797
    return core_ids;
}

// export_components (:804-826): one "#<id>.fa" per component, reads in reader order as
// GenomeReadData::fastX_string (SequenceRecordIterator.h:36-48) + '\n'.
void ClusteringEngine::export_components(const std::vector<ComponentID>& ids, const std::string& dir,
                                         std::ostream& out) const {
    std::filesystem::remove_all(dir);
    std::filesystem::create_directories(dir);
    // one buffered file per component, every read written straight from the record set in read order
    // (the same bytes as building each record's strings: no per-read copies)
    std::map<ComponentID, std::FILE*> files;
    std::vector<ComponentID> owner(reads_.size(), 0);   // 0: in no exported component (ids start at 1)
    std::vector<std::unique_ptr<char[]>> bufs;
    for (ComponentID id : ids) {
        const std::string path = dir + "/#" + std::to_string(id) + ".fa";
        std::FILE* f = std::fopen(path.c_str(), "wb");
        if (!f) throw std::runtime_error("cannot write " + path);
        bufs.emplace_back(new char[1 << 20]);
        std::setvbuf(f, bufs.back().get(), _IOFBF, 1 << 20);
        files[id] = f;
        const auto it = index_.find(id);
        if (it != index_.end())
            for (uint32_t r : it->second.reads)
                if (r >= first_id_ && r - first_id_ < reads_.size()) owner[r - first_id_] = id;
    }
    const bool text = reads_.headers.size() == reads_.size();
    for (uint64_t i = 0; i < reads_.size(); ++i) {
        if (!owner[i]) continue;
        std::FILE* f = files[owner[i]];
        const char* seq = reads_.bases.data() + reads_.offsets[i];
        const size_t len = reads_.offsets[i + 1] - reads_.offsets[i];
        const std::string empty;
        const std::string& hdr = text ? reads_.headers[i] : empty;
        const std::string& qual = text ? reads_.qualities[i] : empty;
        std::fputc(qual.empty() ? '>' : '@', f);
        std::fwrite(hdr.data(), 1, hdr.size(), f);
        std::fputc('\n', f);
        std::fwrite(seq, 1, len, f);
        if (qual.empty()) {
            std::fputc('\n', f);
        } else {
            std::fwrite("\n+\n", 1, 3, f);
            std::fwrite(qual.data(), 1, qual.size(), f);
            std::fputc('\n', f);
        }
    }
    for (auto& kv : files) std::fclose(kv.second);
    out << "Exported " << ids.size() << " components\n";
}

}  // namespace hgah
