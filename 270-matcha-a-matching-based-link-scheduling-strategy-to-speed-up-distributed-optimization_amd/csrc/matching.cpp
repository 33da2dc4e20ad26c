// matching.cpp -- maximum-weight matching for the host-side matching decomposition, without
// networkx.
//
// The reference peels perfect matchings off the base graph with nx.max_weight_matching
// (graph_manager.py:57-83).  WHICH maximum matching comes back decides the schedule, so this is a
// restatement of the algorithm networkx 3.4.2 implements (Edmonds' blossom method in the
// primal-dual form of Galil, "Efficient Algorithms for Finding Maximum Matching in Graphs", ACM
// Computing Surveys 1986; networkx's max_weight_matching), step for step in the same visiting
// orders, so ties break the same way:
//   * vertices are visited in the graph's node order (list(G)), a vertex's neighbours in its
//     adjacency order (G.neighbors) -- the caller passes both (CSR in that order);
//   * the S-vertex queue is a LIFO; blossoms are numbered in creation order and every scan over
//     "blossomparent" / "blossomdual" visits vertices first, then live blossoms by creation;
//   * a blossom's leaves come out of the same explicit-stack walk (children pushed, last popped);
//   * least-slack edge lists keep first-insertion order of the neighbouring blossom;
//   * strict "<" comparisons everywhere a minimum is taken, as networkx does.
// Dual variables are kept doubled, so integer weights stay integer (the reference's graphs are
// unweighted: every weight is 1).  The order in which vertices first become keys of the `mate`
// map is returned too: networkx builds its result set by iterating that dict, and the caller
// rebuilds the identical set (iteration order included) from it.
#include <algorithm>
#include <cstdint>
#include <cstring>
#include <functional>
#include <vector>

#include "mx_common.h"

namespace {

struct Edge {
    int v = -1, w = -1;
    bool none() const { return v < 0; }
};

class Matcher {
   public:
    Matcher(int n, const int64_t* off, const int32_t* adj, const int64_t* wt, bool maxcard)
        : n_(n), off_(off), adj_(adj), wt_(wt), maxcard_(maxcard) {}

    int run(int32_t* mate_out, int32_t* order_out, int* n_order) {
        const int n = n_;
        int64_t maxweight = 0;
        for (int v = 0; v < n; ++v)
            for (int64_t e = off_[v]; e < off_[v + 1]; ++e)
                if (adj_[e] != v && weight_at(e) > maxweight) maxweight = weight_at(e);
        // one slot per vertex and one per blossom ever created (at most n / 2 live at a time,
        // but ids are never reused so that "creation order" is id order)
        grow(n - 1);
        for (int v = 0; v < n; ++v) {
            inblossom_[v] = v;
            parent_[v] = -1;
            base_[v] = v;
            dual_.push_back(maxweight);
        }
        allow_.assign((size_t)n * n, 0);
        mate_.assign(n, -1);
        while (true) {                                   // a stage
            std::fill(label_.begin(), label_.end(), 0);
            for (auto& e : labeledge_) e = Edge{};
            for (auto& e : bestedge_) e = Edge{};
            for (int b = n; b < (int)live_.size(); ++b)
                if (live_[b]) has_mybest_[b] = false;
            std::fill(allow_.begin(), allow_.end(), 0);
            queue_.clear();
            for (int v = 0; v < n; ++v)
                if (mate_[v] < 0 && label_[inblossom_[v]] == 0) assign_label(v, 1, -1);
            bool augmented = false;
            while (true) {                               // a substage
                while (!queue_.empty() && !augmented) {
                    const int v = queue_.back();
                    queue_.pop_back();
                    for (int64_t e = off_[v]; e < off_[v + 1]; ++e) {
                        const int w = adj_[e];
                        if (w == v) continue;
                        const int bv = inblossom_[v], bw = inblossom_[w];
                        if (bv == bw) continue;
                        int64_t kslack = 0;
                        if (!allowed(v, w)) {
                            kslack = slack(v, w);
                            if (kslack <= 0) set_allowed(v, w);
                        }
                        if (allowed(v, w)) {
                            if (label_[bw] == 0) {
                                assign_label(w, 2, v);
                            } else if (label_[bw] == 1) {
                                const int base = scan_blossom(v, w);
                                if (base >= 0) {
                                    add_blossom(base, v, w);
                                } else {
                                    augment_matching(v, w);
                                    augmented = true;
                                    break;
                                }
                            } else if (label_[w] == 0) {
                                label_[w] = 2;
                                labeledge_[w] = Edge{v, w};
                            }
                        } else if (label_[bw] == 1) {
                            if (bestedge_[bv].none() || kslack < slack(bestedge_[bv].v, bestedge_[bv].w))
                                bestedge_[bv] = Edge{v, w};
                        } else if (label_[w] == 0) {
                            if (bestedge_[w].none() || kslack < slack(bestedge_[w].v, bestedge_[w].w))
                                bestedge_[w] = Edge{v, w};
                        }
                    }
                }
                if (augmented) break;
                int deltatype = -1;
                int64_t delta = 0;
                Edge deltaedge;
                int deltablossom = -1;
                if (!maxcard_) {
                    deltatype = 1;
                    delta = *std::min_element(dual_.begin(), dual_.begin() + n);
                }
                for (int v = 0; v < n; ++v) {
                    if (label_[inblossom_[v]] == 0 && !bestedge_[v].none()) {
                        const int64_t d = slack(bestedge_[v].v, bestedge_[v].w);
                        if (deltatype == -1 || d < delta) {
                            delta = d;
                            deltatype = 2;
                            deltaedge = bestedge_[v];
                        }
                    }
                }
                for (int b = 0; b < (int)live_.size(); ++b) {    // vertices, then live blossoms
                    if (!live_[b]) continue;
                    if (parent_[b] == -1 && label_[b] == 1 && !bestedge_[b].none()) {
                        const int64_t kslack = slack(bestedge_[b].v, bestedge_[b].w);
                        const int64_t d = kslack / 2;              // integer weights: kslack is even
                        if (deltatype == -1 || d < delta) {
                            delta = d;
                            deltatype = 3;
                            deltaedge = bestedge_[b];
                        }
                    }
                }
                for (int b = n; b < (int)live_.size(); ++b) {
                    if (!live_[b]) continue;
                    if (parent_[b] == -1 && label_[b] == 2 && (deltatype == -1 || bdual_[b] < delta)) {
                        delta = bdual_[b];
                        deltatype = 4;
                        deltablossom = b;
                    }
                }
                if (deltatype == -1) {                   // max-cardinality optimum reached
                    deltatype = 1;
                    const int64_t m = *std::min_element(dual_.begin(), dual_.begin() + n);
                    delta = m > 0 ? m : 0;
                }
                for (int v = 0; v < n; ++v) {
                    const int l = label_[inblossom_[v]];
                    if (l == 1) dual_[v] -= delta;
                    else if (l == 2) dual_[v] += delta;
                }
                for (int b = n; b < (int)live_.size(); ++b) {
                    if (!live_[b] || parent_[b] != -1) continue;
                    if (label_[b] == 1) bdual_[b] += delta;
                    else if (label_[b] == 2) bdual_[b] -= delta;
                }
                if (deltatype == 1) break;
                if (deltatype == 2 || deltatype == 3) {
                    set_allowed(deltaedge.v, deltaedge.w);
                    queue_.push_back(deltaedge.v);
                } else if (deltatype == 4) {
                    expand_blossom(deltablossom, false);
                }
            }
            for (int v = 0; v < n; ++v)
                if (mate_[v] >= 0 && mate_[mate_[v]] != v) return fail("asymmetric matching");
            if (!augmented) break;
            const int nb = (int)live_.size();            // snapshot: list(blossomdual.keys())
            for (int b = n; b < nb; ++b) {
                if (!live_[b]) continue;
                if (parent_[b] == -1 && label_[b] == 1 && bdual_[b] == 0) expand_blossom(b, true);
            }
        }
        if (err_) return MX_ERR_INVALID;
        for (int v = 0; v < n; ++v) mate_out[v] = mate_[v];
        for (size_t i = 0; i < order_.size(); ++i) order_out[i] = order_[i];
        *n_order = (int)order_.size();
        return MX_OK;
    }

   private:
    int n_;
    const int64_t* off_;
    const int32_t* adj_;
    const int64_t* wt_;
    bool maxcard_;
    bool err_ = false;
    // per vertex / blossom id
    std::vector<int> inblossom_, parent_, base_, label_;
    std::vector<Edge> labeledge_, bestedge_;
    std::vector<char> live_;
    std::vector<int64_t> dual_, bdual_;
    std::vector<std::vector<int>> childs_;
    std::vector<std::vector<Edge>> edges_;
    std::vector<std::vector<Edge>> mybest_;
    std::vector<char> has_mybest_;
    std::vector<uint8_t> allow_;
    std::vector<int> queue_, mate_, order_;
    std::vector<char> in_order_;

    int fail(const char* what) {
        mx::set_error("mx_max_weight_matching: %s", what);
        err_ = true;
        return MX_ERR_INVALID;
    }
    void grow(int id) {                                  // make ids [0, id] valid
        const size_t need = (size_t)id + 1;
        if (inblossom_.size() >= need) return;
        inblossom_.resize(need, -1);
        parent_.resize(need, -1);
        base_.resize(need, -1);
        label_.resize(need, 0);
        labeledge_.resize(need);
        bestedge_.resize(need);
        live_.resize(need, 1);
        bdual_.resize(need, 0);
        childs_.resize(need);
        edges_.resize(need);
        mybest_.resize(need);
        has_mybest_.resize(need, 0);
    }
    bool is_blossom(int b) const { return b >= n_; }
    int64_t weight_at(int64_t e) const { return wt_ ? wt_[e] : 1; }
    int64_t weight(int v, int w) const {
        for (int64_t e = off_[v]; e < off_[v + 1]; ++e)
            if (adj_[e] == w) return weight_at(e);
        return 1;
    }
    int64_t slack(int v, int w) const { return dual_[v] + dual_[w] - 2 * weight(v, w); }
    bool allowed(int v, int w) const { return allow_[(size_t)v * n_ + w] != 0; }
    void set_allowed(int v, int w) { allow_[(size_t)v * n_ + w] = allow_[(size_t)w * n_ + v] = 1; }
    void set_mate(int a, int b) {
        if (!in_order_.size()) in_order_.assign(n_, 0);
        mate_[a] = b;
        if (!in_order_[a]) {
            in_order_[a] = 1;
            order_.push_back(a);
        }
    }
    static int wrap(int j, int len) { return j < 0 ? j + len : j; }   // Python negative index

    // the blossom's leaf vertices: explicit stack, children pushed in order, last popped first
    std::vector<int> leaves(int b) const {
        std::vector<int> out, stack(childs_[b].begin(), childs_[b].end());
        while (!stack.empty()) {
            const int t = stack.back();
            stack.pop_back();
            if (is_blossom(t)) stack.insert(stack.end(), childs_[t].begin(), childs_[t].end());
            else out.push_back(t);
        }
        return out;
    }

    void assign_label(int w, int t, int v) {
        const int b = inblossom_[w];
        label_[w] = label_[b] = t;
        labeledge_[w] = labeledge_[b] = v >= 0 ? Edge{v, w} : Edge{};
        bestedge_[w] = bestedge_[b] = Edge{};
        if (t == 1) {
            if (is_blossom(b)) {
                for (int x : leaves(b)) queue_.push_back(x);
            } else {
                queue_.push_back(b);
            }
        } else if (t == 2) {
            const int base = base_[b];
            assign_label(mate_[base], 1, base);
        }
    }

    int scan_blossom(int v, int w) {
        std::vector<int> path;
        int base = -1;
        while (v >= 0) {
            int b = inblossom_[v];
            if (label_[b] & 4) {
                base = base_[b];
                break;
            }
            path.push_back(b);
            label_[b] = 5;
            if (labeledge_[b].none()) {
                v = -1;
            } else {
                v = labeledge_[b].v;
                b = inblossom_[v];
                v = labeledge_[b].v;
            }
            if (w >= 0) std::swap(v, w);
        }
        for (int b : path) label_[b] = 1;
        return base;
    }

    void add_blossom(int base, int v, int w) {
        const int bb = inblossom_[base];
        int bv = inblossom_[v], bw = inblossom_[w];
        const int b = (int)live_.size();
        grow(b);
        live_[b] = 1;
        base_[b] = base;
        parent_[b] = -1;
        parent_[bb] = b;
        std::vector<int> path;
        std::vector<Edge> edgs{Edge{v, w}};
        while (bv != bb) {
            parent_[bv] = b;
            path.push_back(bv);
            edgs.push_back(labeledge_[bv]);
            v = labeledge_[bv].v;
            bv = inblossom_[v];
        }
        path.push_back(bb);
        std::reverse(path.begin(), path.end());
        std::reverse(edgs.begin(), edgs.end());
        while (bw != bb) {
            parent_[bw] = b;
            path.push_back(bw);
            edgs.push_back(Edge{labeledge_[bw].w, labeledge_[bw].v});
            w = labeledge_[bw].v;
            bw = inblossom_[w];
        }
        childs_[b] = path;
        edges_[b] = edgs;
        label_[b] = 1;
        labeledge_[b] = labeledge_[bb];
        bdual_[b] = 0;
        for (int x : leaves(b)) {
            if (label_[inblossom_[x]] == 2) queue_.push_back(x);
            inblossom_[x] = b;
        }
        // least-slack edges to neighbouring S-blossoms, keyed in first-insertion order
        std::vector<int> keys;
        std::vector<Edge> vals;
        std::vector<int> slot(live_.size(), -1);
        for (int sub : childs_[b]) {
            std::vector<Edge> nblist;
            if (is_blossom(sub)) {
                if (has_mybest_[sub]) {
                    nblist = mybest_[sub];
                    has_mybest_[sub] = 0;
                    mybest_[sub].clear();
                } else {
                    for (int x : leaves(sub))
                        for (int64_t e = off_[x]; e < off_[x + 1]; ++e)
                            if (adj_[e] != x) nblist.push_back(Edge{x, adj_[e]});
                }
            } else {
                for (int64_t e = off_[sub]; e < off_[sub + 1]; ++e)
                    if (adj_[e] != sub) nblist.push_back(Edge{sub, adj_[e]});
            }
            for (const Edge& k : nblist) {
                int i = k.v, j = k.w;
                if (inblossom_[j] == b) std::swap(i, j);
                const int bj = inblossom_[j];
                if (bj != b && label_[bj] == 1 &&
                    (slot[bj] < 0 || slack(i, j) < slack(vals[slot[bj]].v, vals[slot[bj]].w))) {
                    if (slot[bj] < 0) {
                        slot[bj] = (int)keys.size();
                        keys.push_back(bj);
                        vals.push_back(k);
                    } else {
                        vals[slot[bj]] = k;
                    }
                }
            }
            bestedge_[sub] = Edge{};
        }
        mybest_[b] = vals;
        has_mybest_[b] = 1;
        Edge best;
        int64_t bestslack = 0;
        for (const Edge& k : mybest_[b]) {
            const int64_t ks = slack(k.v, k.w);
            if (best.none() || ks < bestslack) {
                best = k;
                bestslack = ks;
            }
        }
        bestedge_[b] = best;
    }

    void expand_blossom(int b, bool endstage) {
        for (int s : childs_[b]) {
            parent_[s] = -1;
            if (is_blossom(s)) {
                if (endstage && bdual_[s] == 0) {
                    expand_blossom(s, endstage);
                } else {
                    for (int x : leaves(s)) inblossom_[x] = s;
                }
            } else {
                inblossom_[s] = s;
            }
        }
        if (!endstage && label_[b] == 2) {
            const std::vector<int>& ch = childs_[b];
            const std::vector<Edge>& ed = edges_[b];
            const int L = (int)ch.size();
            const int entrychild = inblossom_[labeledge_[b].w];
            int j = (int)(std::find(ch.begin(), ch.end(), entrychild) - ch.begin());
            int jstep;
            if (j & 1) {
                j -= L;
                jstep = 1;
            } else {
                jstep = -1;
            }
            int v = labeledge_[b].v, w = labeledge_[b].w;
            while (j != 0) {
                int p, q;
                if (jstep == 1) {
                    p = ed[wrap(j, L)].v;
                    q = ed[wrap(j, L)].w;
                } else {
                    q = ed[wrap(j - 1, L)].v;
                    p = ed[wrap(j - 1, L)].w;
                }
                label_[w] = 0;
                label_[q] = 0;
                assign_label(w, 2, v);
                set_allowed(p, q);
                j += jstep;
                if (jstep == 1) {
                    v = ed[wrap(j, L)].v;
                    w = ed[wrap(j, L)].w;
                } else {
                    w = ed[wrap(j - 1, L)].v;
                    v = ed[wrap(j - 1, L)].w;
                }
                set_allowed(v, w);
                j += jstep;
            }
            const int bw = ch[wrap(j, L)];
            label_[w] = label_[bw] = 2;
            labeledge_[w] = labeledge_[bw] = Edge{v, w};
            bestedge_[bw] = Edge{};
            j += jstep;
            while (ch[wrap(j, L)] != entrychild) {
                const int bv = ch[wrap(j, L)];
                if (label_[bv] == 1) {
                    j += jstep;
                    continue;
                }
                int x = bv;
                if (is_blossom(bv)) {
                    for (int leaf : leaves(bv)) {                // x: first labelled leaf, else the last
                        x = leaf;
                        if (label_[leaf]) break;
                    }
                }
                if (label_[x]) {
                    label_[x] = 0;
                    label_[mate_[base_[bv]]] = 0;
                    assign_label(x, 2, labeledge_[x].v);
                }
                j += jstep;
            }
        }
        label_[b] = 0;
        labeledge_[b] = Edge{};
        bestedge_[b] = Edge{};
        live_[b] = 0;
        parent_[b] = -1;
        bdual_[b] = 0;
    }

    void augment_blossom(int b, int v) {
        int t = v;
        while (parent_[t] != b) t = parent_[t];
        if (is_blossom(t)) augment_blossom(t, v);
        std::vector<int>& ch = childs_[b];
        std::vector<Edge>& ed = edges_[b];
        const int L = (int)ch.size();
        const int i = (int)(std::find(ch.begin(), ch.end(), t) - ch.begin());
        int j = i, jstep;
        if (i & 1) {
            j -= L;
            jstep = 1;
        } else {
            jstep = -1;
        }
        while (j != 0) {
            j += jstep;
            t = ch[wrap(j, L)];
            int w, x;
            if (jstep == 1) {
                w = ed[wrap(j, L)].v;
                x = ed[wrap(j, L)].w;
            } else {
                x = ed[wrap(j - 1, L)].v;
                w = ed[wrap(j - 1, L)].w;
            }
            if (is_blossom(t)) augment_blossom(t, w);
            j += jstep;
            t = ch[wrap(j, L)];
            if (is_blossom(t)) augment_blossom(t, x);
            set_mate(w, x);
            set_mate(x, w);
        }
        std::rotate(ch.begin(), ch.begin() + i, ch.end());
        std::rotate(ed.begin(), ed.begin() + i, ed.end());
        base_[b] = base_[ch[0]];
    }

    void augment_matching(int v, int w) {
        const int pairs[2][2] = {{v, w}, {w, v}};
        for (const auto& pr : pairs) {
            int s = pr[0], j = pr[1];
            while (true) {
                const int bs = inblossom_[s];
                if (is_blossom(bs)) augment_blossom(bs, s);
                set_mate(s, j);
                if (labeledge_[bs].none()) break;
                const int t = labeledge_[bs].v;
                const int bt = inblossom_[t];
                s = labeledge_[bt].v;
                j = labeledge_[bt].w;
                if (is_blossom(bt)) augment_blossom(bt, j);
                set_mate(j, s);
            }
        }
    }
};

}  // namespace

extern "C" int mx_max_weight_matching(int n, const int64_t* adj_off, const int32_t* adj, const int64_t* adj_w,
                                      int maxcardinality, int32_t* mate_out, int32_t* order_out, int* n_order) {
    MX_CHECK(n >= 0 && (n == 0 || (adj_off && mate_out && order_out && n_order)), "mx_max_weight_matching: bad arguments");
    if (n == 0) {
        if (n_order) *n_order = 0;
        return MX_OK;
    }
    MX_CHECK(adj_off[0] == 0 && (adj_off[n] == 0 || adj), "mx_max_weight_matching: bad adjacency offsets");
    MX_CHECK(n <= 1 << 15, "mx_max_weight_matching: %d nodes (at most 32768)", n);
    for (int v = 0; v < n; ++v) {
        MX_CHECK(adj_off[v + 1] >= adj_off[v], "mx_max_weight_matching: offsets not ascending at %d", v);
        for (int64_t e = adj_off[v]; e < adj_off[v + 1]; ++e)
            MX_CHECK(adj[e] >= 0 && adj[e] < n, "mx_max_weight_matching: neighbour %d of %d out of range", adj[e], v);
    }
    Matcher m(n, adj_off, adj, adj_w, maxcardinality != 0);
    return m.run(mate_out, order_out, n_order);
}
