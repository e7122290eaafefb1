// driver.cpp - exercises the multi-threaded host graph builder (csrc/graph_host.cpp)
// outside Python, so that it can run under AddressSanitizer + UBSan and under
// ThreadSanitizer (scripts/sanitize_host.sh).  Every result is also checked
// against a serial restatement written here, so the run is a test as well.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <map>
#include <random>
#include <vector>

#include "igr.h"

#define CHECK(cond)                                                              \
    do {                                                                         \
        if (!(cond)) {                                                           \
            std::fprintf(stderr, "%s:%d: CHECK failed: %s (%s)\n", __FILE__, __LINE__, #cond, igr_last_error()); \
            std::exit(1);                                                        \
        }                                                                        \
    } while (0)

struct Csr {
    std::vector<int64_t> row_ptr, eid;
    std::vector<int32_t> col;
    std::vector<float> val;
    int64_t nnz = 0;
};

static Csr build(int64_t nr, int64_t nc, const std::vector<int64_t> &r, const std::vector<int64_t> &c,
                 const std::vector<float> &v, int dedup, int threads) {
    Csr g;
    const int64_t n = (int64_t)r.size();
    g.row_ptr.resize(nr + 1);
    g.col.resize(std::max<int64_t>(n, 1));
    g.val.resize(std::max<int64_t>(n, 1));
    g.eid.resize(std::max<int64_t>(n, 1));
    CHECK(igr_csr_from_coo(nr, nc, n, r.data(), c.data(), v.data(), dedup, g.row_ptr.data(), g.col.data(),
                           g.val.data(), g.eid.data(), &g.nnz, threads) == IGR_OK);
    g.col.resize(g.nnz);
    g.val.resize(g.nnz);
    g.eid.resize(g.nnz);
    return g;
}

static void one_case(int64_t nr, int64_t nc, int64_t n, unsigned seed) {
    std::mt19937_64 rng(seed);
    std::vector<int64_t> r(n), c(n);
    std::vector<float> v(n);
    for (int64_t i = 0; i < n; ++i) {
        // skewed rows (hub rows get long buckets), many duplicate pairs
        const double u = std::generate_canonical<double, 53>(rng);
        r[i] = std::min<int64_t>(nr - 1, (int64_t)(nr * u * u * u));
        c[i] = (int64_t)(rng() % (uint64_t)nc);
        v[i] = (float)((int)(rng() % 7) - 3);
    }
    for (int dedup = 0; dedup <= 1; ++dedup) {
        const Csr a = build(nr, nc, r, c, v, dedup, 1), b = build(nr, nc, r, c, v, dedup, 8);
        CHECK(a.nnz == b.nnz && a.row_ptr == b.row_ptr && a.col == b.col && a.val == b.val && a.eid == b.eid);
        // serial restatement: (row, col) -> summed value / first position
        std::map<std::pair<int64_t, int64_t>, std::pair<float, int64_t>> m;
        if (dedup) {
            for (int64_t i = 0; i < n; ++i) {
                auto it = m.find({r[i], c[i]});
                if (it == m.end()) m[{r[i], c[i]}] = {v[i], i};
                else it->second.first += v[i];
            }
            CHECK((int64_t)m.size() == a.nnz);
            int64_t p = 0;
            for (auto &kv : m) {
                CHECK(a.col[p] == kv.first.second && a.val[p] == kv.second.first && a.eid[p] == kv.second.second);
                CHECK(a.row_ptr[kv.first.first] <= p && p < a.row_ptr[kv.first.first + 1]);
                ++p;
            }
        } else {
            CHECK(a.nnz == n);
            for (int64_t p = 0; p < n; ++p) CHECK(a.col[p] == c[a.eid[p]] && a.val[p] == v[a.eid[p]]);
            for (int64_t row = 0; row < nr; ++row)
                for (int64_t p = a.row_ptr[row]; p < a.row_ptr[row + 1]; ++p) {
                    CHECK(r[a.eid[p]] == row);
                    if (p > a.row_ptr[row])
                        CHECK(a.col[p - 1] < a.col[p] || (a.col[p - 1] == a.col[p] && a.eid[p - 1] < a.eid[p]));
                }
        }
        // transpose, 1 thread vs 8
        std::vector<int64_t> trp1(nc + 1), trp8(nc + 1), tp1(std::max<int64_t>(a.nnz, 1)), tp8(tp1.size());
        std::vector<int32_t> tc1(tp1.size()), tc8(tp1.size());
        CHECK(igr_csr_transpose(nr, nc, a.row_ptr.data(), a.col.data(), trp1.data(), tc1.data(), tp1.data(), 1) == 0);
        CHECK(igr_csr_transpose(nr, nc, a.row_ptr.data(), a.col.data(), trp8.data(), tc8.data(), tp8.data(), 8) == 0);
        CHECK(trp1 == trp8 && tc1 == tc8 && tp1 == tp8);
        for (int64_t cc = 0; cc < nc; ++cc)
            for (int64_t q = trp1[cc]; q < trp1[cc + 1]; ++q) {
                CHECK(a.col[tp1[q]] == cc);
                CHECK(a.row_ptr[tc1[q]] <= tp1[q] && tp1[q] < a.row_ptr[tc1[q] + 1]);
            }
        // row sums and symmetric normalisation values
        std::vector<float> rs(nr), dr(nr), dc(nc), out(std::max<int64_t>(a.nnz, 1));
        CHECK(igr_csr_row_sums(nr, a.row_ptr.data(), a.val.data(), rs.data()) == 0);
        for (int64_t row = 0; row < nr; ++row) {
            float s = 0.f;
            for (int64_t p = a.row_ptr[row]; p < a.row_ptr[row + 1]; ++p) s += a.val[p];
            CHECK(rs[row] == s);
            dr[row] = 1.f / (1.f + (float)(row % 5));
        }
        for (int64_t cc = 0; cc < nc; ++cc) dc[cc] = 1.f / (2.f + (float)(cc % 3));
        CHECK(igr_sym_norm_values(nr, a.row_ptr.data(), a.col.data(), a.val.data(), dr.data(), dc.data(), out.data()) == 0);
        for (int64_t row = 0; row < nr; ++row)
            for (int64_t p = a.row_ptr[row]; p < a.row_ptr[row + 1]; ++p)
                CHECK(out[p] == (dr[row] * a.val[p]) * dc[a.col[p]]);
        // row schedule: every row exactly once, chunks cover the long rows
        int64_t no = 0, ns = 0, nch = 0;
        CHECK(igr_plan_size(nr, a.row_ptr.data(), 64, 64, &no, &ns, &nch) == 0);
        CHECK(no + ns == nr);
        std::vector<int32_t> order(std::max<int64_t>(no, 1)), srow(std::max<int64_t>(ns, 1)), crow(std::max<int64_t>(nch, 1));
        std::vector<int64_t> sptr(ns + 1), cbeg(std::max<int64_t>(nch, 1));
        CHECK(igr_plan_fill(nr, a.row_ptr.data(), 64, 64, 1024, order.data(), srow.data(), sptr.data(), crow.data(),
                            cbeg.data()) == 0);
        std::vector<int> seen(nr, 0);
        for (int64_t i = 0; i < no; ++i) seen[order[i]]++;
        for (int64_t s = 0; s < ns; ++s) {
            seen[srow[s]]++;
            int64_t covered = 0;
            for (int64_t k = sptr[s]; k < sptr[s + 1]; ++k) {
                CHECK(crow[k] == srow[s] && cbeg[k] == a.row_ptr[srow[s]] + covered);
                covered += 64;
            }
            CHECK(covered >= a.row_ptr[srow[s] + 1] - a.row_ptr[srow[s]]);
        }
        for (int64_t row = 0; row < nr; ++row) CHECK(seen[row] == 1);
    }
    // the shard set-up passes: occurrences of each id, and the pairs of one id range in stream order
    for (int nt : {1, 8}) {
        std::vector<int64_t> cnt(nr, -1), ref(nr, 0);
        CHECK(igr_count_ids(n, r.data(), nr, cnt.data(), nt) == 0);
        for (int64_t i = 0; i < n; ++i) ref[r[i]]++;
        CHECK(cnt == ref);
        const int64_t lo = nr / 4, hi = nr / 4 + std::max<int64_t>(1, nr / 2);
        int64_t m = -1;
        CHECK(igr_select_id_range(n, r.data(), c.data(), lo, hi, nullptr, nullptr, &m, nt) == 0);
        std::vector<int64_t> ok(std::max<int64_t>(m, 1)), oo(std::max<int64_t>(m, 1));
        int64_t m2 = -1;
        CHECK(igr_select_id_range(n, r.data(), c.data(), lo, hi, ok.data(), oo.data(), &m2, nt) == 0);
        CHECK(m2 == m);
        int64_t j = 0;
        for (int64_t i = 0; i < n; ++i)
            if (r[i] >= lo && r[i] < hi) {
                CHECK(j < m && ok[j] == r[i] - lo && oo[j] == c[i]);
                ++j;
            }
        CHECK(j == m);
    }
    {
        std::vector<int64_t> bad = r, cnt(nr);
        bad[n - 1] = nr;
        CHECK(igr_count_ids(n, bad.data(), nr, cnt.data(), 8) == IGR_ERR_ARG);
    }
    // error path: an out-of-range index is refused with a message
    std::vector<int64_t> rb = r, rp(nr + 1);
    std::vector<int32_t> cb(n);
    rb[n / 2] = nr;
    int64_t k = 0;
    CHECK(igr_csr_from_coo(nr, nc, n, rb.data(), c.data(), nullptr, 1, rp.data(), cb.data(), nullptr, nullptr, &k, 8) ==
          IGR_ERR_ARG);
    CHECK(igr_last_error()[0] != 0);
}

int main() {
    one_case(5000, 3000, 200000, 1);   // multi-threaded path (>= 4096 items per loop)
    one_case(7, 5, 13, 2);             // tiny: serial path, empty rows
    one_case(300, 40000, 150000, 3);   // few long rows, wide
    one_case(100000, 10, 120000, 4);   // many rows, few columns: heavy duplicate merging
    std::puts("host graph builder: all checks passed");
    return 0;
}
