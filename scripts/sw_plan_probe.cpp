// Host-phase timing of fecgpu_sw_decode's plan on the bench.py --config 7
// pattern (524,288 sources, a repair every 8 over the last 32, 2 % i.i.d.
// loss of sources and repairs; also 5 % and bursts): header checks, then the
// plan (status/lost scan + sweep) on the caller alone and on the helper pool,
// whose output must equal the serial plan's array for array.  Compiles the
// library's own fec_sw.cpp into the probe (its helpers are file-local); no
// GPU call.  Median of 50 runs (argv: [threads [runs]]).
#include "../quic-fec-eps_amd/csrc/fec_sw.cpp"

#include <chrono>
#include <cstdio>
#include <random>

using clk = std::chrono::steady_clock;

static double med(std::vector<double> v) {
    std::sort(v.begin(), v.end());
    return v[v.size() / 2];
}

struct Copy {  // the arrays a plan hands the GPU
    std::vector<uint8_t> comps, unk, eqr, eqc, eqh, st;
    uint64_t amat, nsolve, tcoef;
    int max_nss, max_p;
    bool operator==(const Copy &o) const {
        return comps == o.comps && unk == o.unk && eqr == o.eqr && eqc == o.eqc && eqh == o.eqh && st == o.st &&
               amat == o.amat && nsolve == o.nsolve && tcoef == o.tcoef && max_nss == o.max_nss && max_p == o.max_p;
    }
};

int main(int argc, char **argv) {
    const uint64_t nrep = 65536, k = 8, W = 32, nsrc = nrep * k;
    std::vector<fecgpu_sw_repair> hdr(nrep);
    for (uint64_t t = 0; t < nrep; t++) {
        const uint64_t end = (t + 1) * k, fss = end > W ? end - W : 0;
        hdr[t] = fecgpu_sw_repair{fss, (uint16_t)(end - fss), (uint16_t)(t & 0xffff), 15, {0, 0, 0}};
    }
    const int threads = argc > 1 ? std::atoi(argv[1]) : 0;
    const int reps = argc > 2 ? std::max(1, std::atoi(argv[2])) : 50;
    std::vector<uint8_t> pin;
    auto host = [&](size_t bytes, void **p) -> ssize_t {
        if (pin.size() < bytes) pin.resize(bytes);
        *p = pin.data();
        return 0;
    };
    bool all_equal = true;
    for (int pattern = 0; pattern < 3; pattern++) {
        std::mt19937_64 g(1 + pattern);
        std::uniform_real_distribution<double> U(0, 1);
        std::vector<uint8_t> sp(nsrc), rp(nrep), st(nsrc);
        const double loss = pattern == 1 ? 0.05 : 0.02;
        for (auto &x : sp) x = U(g) >= loss;
        for (auto &x : rp) x = U(g) >= loss;
        if (pattern == 2)  // bursts of 20 every 4096 sources on top
            for (uint64_t b = 100; b + 20 < nsrc; b += 4096)
                for (int j = 0; j < 20; j++) sp[b + j] = 0;
        std::vector<double> th, t1s, tps;
        Copy ref{}, got{};
        uint64_t nlost = 0, ncomp = 0, neq = 0;
        for (int rep = 0; rep < reps; rep++) {
            const auto t0 = clk::now();
            uint64_t wmax = 1, prev = 0;
            for (uint64_t t = 0; t < nrep; t++) {
                if (!header_ok(hdr[t], nsrc) || hdr[t].fss < prev) return 1;
                prev = hdr[t].fss;
                wmax = std::max<uint64_t>(wmax, hdr[t].nss);
            }
            const auto t1 = clk::now();
            for (int mode = 0; mode < 2; mode++) {
                SwPlan &P = sw_plan_scratch();
                SwLayout L{};
                const auto a = clk::now();
                const ssize_t nl = sw_plan(host, sp.data(), nsrc, st.data(), rp.data(), hdr.data(), nrep, wmax, P, L,
                                           mode == 0 ? 1 : threads);
                const auto b = clk::now();
                if (nl < 0) return 2;
                (mode == 0 ? t1s : tps).push_back(std::chrono::duration<double, std::micro>(b - a).count());
                Copy &c = mode == 0 ? ref : got;
                auto bytes = [](const void *p, size_t n) {
                    const uint8_t *q = static_cast<const uint8_t *>(p);
                    return std::vector<uint8_t>(q, q + n);
                };
                c.comps = bytes(P.comps, P.ncomp * sizeof(SwComp));
                c.unk = bytes(P.unk, P.nunk * 8);
                c.eqr = bytes(P.eqr, P.neq * 8);
                c.eqc = bytes(P.eqc, P.neq * 4);
                c.eqh = bytes(P.eqh, P.neq * sizeof(fecgpu_sw_repair));
                c.st = st;
                c.amat = P.amat;
                c.nsolve = P.nsolve;
                c.tcoef = P.tcoef;
                c.max_nss = P.max_nss;
                c.max_p = P.max_p;
                nlost = (uint64_t)nl;
                ncomp = P.ncomp;
                neq = P.neq;
            }
            if (!(ref == got)) all_equal = false;
            th.push_back(std::chrono::duration<double, std::micro>(t1 - t0).count());
        }
        std::printf("{\"pattern\": \"%s\", \"threads\": %d, \"nsrc\": %lu, \"lost\": %lu, \"systems\": %lu, "
                    "\"equations\": %lu, \"us_headers\": %.1f, \"us_plan_serial\": %.1f, \"us_plan_pool\": %.1f, "
                    "\"equal\": %s}\n",
                    pattern == 0 ? "iid 2%" : pattern == 1 ? "iid 5%" : "iid 2% + bursts of 20",
                    threads ? std::min(threads, PlanPool::get().size()) : PlanPool::get().size(), (unsigned long)nsrc,
                    (unsigned long)nlost, (unsigned long)ncomp, (unsigned long)neq, med(th), med(t1s), med(tps),
                    all_equal ? "true" : "false");
    }
    return all_equal ? 0 : 3;
}
