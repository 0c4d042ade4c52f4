// sdig_host.cpp -- host side of the Brakedown / SDIG encoding: code parameters, dimensions and
// matrix generation (lcpc-brakedown-pc/src/{codespec.rs, lib.rs, matgen.rs}).
//
// Matrix generation is sequential within a level (one ChaCha20 stream per level, matgen.rs:
// 41-46) and independent across levels, so levels are generated on their own host threads.
// The sparse matrices are converted to output-major (CSR) form for the device gathers.
#include "sdig.hpp"

#include <algorithm>
#include <cmath>
#include <thread>

#include "transcript.hpp"

namespace lcpc {

namespace {

const SdigSpec k_specs[7] = {
    {0, 0, 0, 0, 0, 0, 0},
    {239, 2000, 71, 2500, 71, 50, 20},    // SdigCode1 codespec.rs:169-177
    {69, 500, 111, 2500, 147, 100, 20},   // SdigCode2 :180-188
    {89, 500, 61, 1000, 1521, 1000, 20},  // SdigCode3 :191-199 (the default, lib.rs:19)
    {1, 5, 41, 500, 41, 25, 20},          // SdigCode4 :202-210
    {211, 1000, 97, 1000, 202, 125, 20},  // SdigCode5 :213-221
    {119, 500, 241, 2000, 43, 25, 20},    // SdigCode6 :224-232
};

double ent(double z) {  // codespec.rs:17-21
  const double m = 1.0 - z;
  return -z * std::log2(z) - m * std::log2(m);
}

struct Derived {  // SdigSpecification's f64 helpers (codespec.rs:84-135)
  double alpha, beta, r, mu, nu, cn1, cn2, dn1, dn2;
  explicit Derived(const SdigSpec &s) {
    alpha = (double)s.an / (double)s.ad;
    beta = (double)s.bn / (double)s.bd;
    r = (double)s.rn / (double)s.rd;
    mu = r - 1.0 - r * alpha;
    nu = beta + alpha * beta + 0.03;
    cn1 = ent(beta) + alpha * ent(1.28 * beta / alpha);
    cn2 = beta * std::log2(alpha / (1.28 * beta));
    dn1 = r * alpha * ent(beta / r) + mu * ent(nu / mu);
    dn2 = alpha * beta * std::log2(mu / nu);
  }
};

size_t ceil_muldiv(size_t n, size_t num, size_t den) { return (n * num + den - 1) / den; }

size_t next_pow2(size_t v) {
  size_t p = 1;
  while (p < v) p <<= 1;
  return p;
}
size_t log2_np2(size_t v) {
  size_t p = next_pow2(v), l = 0;
  while (((size_t)1 << l) < p) l++;
  return l;
}
// lcpc-2d n_degree_tests (lib.rs:642-645)
size_t n_degree_tests(size_t lambda, size_t len, size_t flog2) {
  const size_t den = flog2 - log2_np2(len);
  return (lambda + den - 1) / den;
}

// SdigEncodingS::_new_from_np1 (lib.rs:69-99): pick np1 or np1 / 2
size_t choose_np(int code, int num_bits, size_t len, size_t np1) {
  if (np1 > len) np1 = len;
  const size_t nco = sdig_n_col_opens(code);
  const size_t flog2 = (size_t)num_bits - 1;
  const size_t nr1 = (len + np1 - 1) / np1;
  const size_t nd1 = n_degree_tests(128, np1 * 2, flog2);
  const size_t np2 = np1 / 2;
  if (np2 == 0) return np1;
  const size_t nr2 = (len + np2 - 1) / np2;
  const size_t nd2 = n_degree_tests(128, np2 * 2, flog2);
  const size_t sz1 = nco * nr1 + (1 + nd1) * np1;
  const size_t sz2 = nco * nr2 + (1 + nd2) * np2;
  return sz1 < sz2 ? np1 : np2;
}

// matgen::gen_code (matgen.rs:114-188) -> CSC, then transposed to CSR
void gen_code(int limbs, int num_bits, const uint64_t *p, size_t n, size_t m, size_t d,
              ChaCha20Rng &rng, CsrHost &out) {
  std::vector<uint32_t> col_rows;  // CSC row indices, d per column (distinct by construction)
  std::vector<uint64_t> col_vals;
  col_rows.reserve(n * d);
  col_vals.reserve(n * d * limbs);
  std::vector<size_t> tmp;
  tmp.reserve(d);
  uint64_t v[4];
  for (size_t c = 0; c < n; c++) {
    tmp.clear();
    // sample_iter(Uniform(0, m)).filter(unseen).take(d)
    while (tmp.size() < d) {
      const size_t x = (size_t)uniform_usize(rng, 0, m);
      if (std::find(tmp.begin(), tmp.end(), x) == tmp.end()) tmp.push_back(x);
    }
    std::sort(tmp.begin(), tmp.end());
    for (size_t x : tmp) {
      // F::random until nonzero (matgen.rs:171-177)
      for (;;) {
        field_random(rng, limbs, num_bits, p, v, 1);
        uint64_t nz = 0;
        for (int l = 0; l < limbs; l++) nz |= v[l];
        if (nz) break;
      }
      col_rows.push_back((uint32_t)x);
      for (int l = 0; l < limbs; l++) col_vals.push_back(v[l]);
    }
  }
  // CSC (column c owns entries [c*d, (c+1)*d)) -> CSR
  out.rows = m;
  out.cols = n;
  out.ptr.assign(m + 1, 0);
  for (uint32_t r : col_rows) out.ptr[r + 1]++;
  for (size_t r = 0; r < m; r++) out.ptr[r + 1] += out.ptr[r];
  out.idx.resize(col_rows.size());
  out.val.resize(col_rows.size() * limbs);
  std::vector<uint32_t> fill(out.ptr.begin(), out.ptr.end() - 1);
  for (size_t c = 0; c < n; c++)
    for (size_t k = c * d; k < (c + 1) * d; k++) {
      const uint32_t r = col_rows[k];
      const uint32_t dst = fill[r]++;
      out.idx[dst] = (uint32_t)c;
      for (int l = 0; l < limbs; l++) out.val[(size_t)dst * limbs + l] = col_vals[k * limbs + l];
    }
}

}  // namespace

const SdigSpec *sdig_spec(int code) { return code >= 1 && code <= 6 ? &k_specs[code] : nullptr; }

size_t sdig_n_col_opens(int code) {
  const SdigSpec *s = sdig_spec(code);
  if (!s) return 0;
  // dist = beta / r (codespec.rs:44-48); -LAMBDA / log2(1 - dist / 3)
  const double dist = (double)(s->bn * s->rd) / (double)(s->bd * s->rn);
  return (size_t)std::ceil(-128.0 / std::log2(1.0 - dist / 3.0));
}

size_t sdig_new_np(int code, int num_bits, size_t len) {
  if (!sdig_spec(code) || len == 0) return 0;
  const double lncf = (double)(sdig_n_col_opens(code) * len);
  const double ndt =
      (double)n_degree_tests(128, (size_t)std::ceil(std::sqrt(lncf)) * 2, (size_t)num_bits - 1);
  const size_t np1 = (size_t)std::ceil(std::sqrt(lncf / ndt));
  return choose_np(code, num_bits, len, np1);
}

size_t sdig_new_ml_np(int code, int num_bits, size_t n_vars) {
  if (!sdig_spec(code) || n_vars >= 63) return 0;
  const size_t n_mon = (size_t)1 << n_vars;
  const double lncf = (double)(sdig_n_col_opens(code) * n_mon);
  const double ndt =
      (double)n_degree_tests(128, (size_t)std::ceil(std::sqrt(lncf)) * 2, (size_t)num_bits - 1);
  const size_t np1 = next_pow2((size_t)std::ceil(std::sqrt(lncf / ndt)));
  return choose_np(code, num_bits, n_mon, np1);
}

int sdig_level_dims(int code, size_t n, double log2p, std::vector<std::array<size_t, 3>> &pre,
                    std::vector<std::array<size_t, 3>> &post) {
  const SdigSpec *s = sdig_spec(code);
  pre.clear();
  post.clear();
  if (!s || !(n > s->blen)) return -1;
  const Derived dv(*s);
  std::vector<size_t> chain;
  for (size_t ni = n; ni > s->blen; ni = ceil_muldiv(ni, s->an, s->ad)) chain.push_back(ni);
  chain.push_back(ceil_muldiv(chain.back(), s->an, s->ad));
  const int nlev = (int)chain.size() - 1;
  if (nlev < 1) return -1;
  for (int i = 0; i < nlev; i++) {
    const size_t ni = chain[i], mi = chain[i + 1];
    const size_t a = ceil_muldiv(ni, 32 * s->bn, 25 * s->bd);
    const size_t b = 4 + ceil_muldiv(ni, s->bn, s->bd);
    const size_t c = (size_t)std::ceil((110.0 / (double)ni + dv.cn1) / dv.cn2);
    const size_t cn = std::min(std::min(std::max(a, b), c), mi);
    pre.push_back({ni, mi, cn});
    const size_t nip = ceil_muldiv(mi, s->rn, s->rd);
    const size_t mip = ceil_muldiv(ni, s->rn, s->rd) - ni - nip;
    const size_t t1 = ceil_muldiv(ni, 2 * s->bn, s->bd);
    const size_t t2 = ceil_muldiv(ni, s->rn, s->rd) - ni + 110;
    size_t dn = std::min(t1 + (size_t)std::ceil((double)t2 / log2p),
                         (size_t)std::ceil((110.0 / (double)ni + dv.dn1) / dv.dn2));
    dn = std::min(dn, mip);
    post.push_back({nip, mip, dn});
  }
  return nlev;
}

bool sdig_generate(int limbs, int num_bits, const uint64_t *p, int code, size_t n, uint64_t seed,
                   std::vector<CsrHost> &pre, std::vector<CsrHost> &post) {
  std::vector<std::array<size_t, 3>> pd, qd;
  const int nlev = sdig_level_dims(code, n, (double)(num_bits - 1), pd, qd);
  if (nlev < 1) return false;
  pre.assign(nlev, CsrHost{});
  post.assign(nlev, CsrHost{});
  auto level = [&](int i) {
    // matgen.rs:41-46: seed_from_u64(seed), set_stream(i), precode then postcode
    ChaCha20Rng rng = ChaCha20Rng::seed_from_u64(seed);
    rng.set_stream((uint64_t)i);
    gen_code(limbs, num_bits, p, pd[i][0], pd[i][1], pd[i][2], rng, pre[i]);
    gen_code(limbs, num_bits, p, qd[i][0], qd[i][1], qd[i][2], rng, post[i]);
  };
  std::vector<std::thread> th;
  for (int i = 1; i < nlev; i++) th.emplace_back(level, i);
  level(0);
  for (auto &t : th) t.join();
  return true;
}

size_t sdig_codeword_length(const std::vector<CsrHost> &pre, const std::vector<CsrHost> &post) {
  size_t len = pre[0].cols + post.back().cols;
  for (size_t i = 0; i + 1 < pre.size(); i++) len += pre[i].rows;
  for (const auto &q : post) len += q.rows;
  return len;
}

}  // namespace lcpc
