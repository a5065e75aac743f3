// Host-only timing of the agent's per-actor walk (run_actor_walk, agent.cpp) on the mixed agent
// call's shape (bench.py agent_e2e_mixed): 1000 actors x 1049 versions, ~5 % of the versions as two
// partial halves (second halves later in the call) and ~10 % of those re-sent whole -- the changesets
// the device header passes leave to the host; every other version a device-decided run. No GPU: the
// walk touches only host state. Build: tools/walkbench/build.sh; run: ./walk_bench [reps] [serial].
#include "../../corrosion_amd/csrc/agent.cpp"

#include <random>

using namespace corro;

int main(int argc, char **argv) {
    const int reps = argc > 1 ? std::atoi(argv[1]) : 20;
    const bool serial = argc > 2 && std::atoi(argv[2]) != 0;
    const uint32_t NA = 1000, NV = 1049;
    std::mt19937_64 rng(5);
    std::uniform_real_distribution<double> U(0, 1);
    std::vector<corro_changeset> cs;
    std::vector<std::vector<uint64_t>> idx(NA);
    std::vector<std::vector<uint64_t>> rs(NA), re(NA);
    std::vector<ActorId> ids(NA);
    for (uint32_t a = 0; a < NA; a++) {
        for (int b = 0; b < 16; b++) ids[a][b] = (uint8_t)((a * 131 + b * 7) & 0xFF);
        ids[a][0] = (uint8_t)(a >> 8);
        ids[a][1] = (uint8_t)a;
        std::vector<uint64_t> tail;
        uint64_t run0 = 0;
        auto close_run = [&](uint64_t v) {  // versions [run0, v) decided on the device
            if (run0 && run0 < v) {
                rs[a].push_back(run0);
                re[a].push_back(v - 1);
            }
            run0 = 0;
        };
        for (uint64_t v = 1; v <= NV; v++) {
            const double u = U(rng);
            const uint64_t cnt = 64;
            corro_changeset c{};
            c.actor_id = ids[a].data();
            c.site = a;
            c.kind = CORRO_CS_FULL;
            c.version_start = c.version_end = v;
            c.last_seq = cnt - 1;
            c.ts = (v << 32) | a;
            c.change_off = ((uint64_t)a * NV + v) * cnt;
            if (u >= 0.05 && u < 0.10) {  // two partial halves, the second later; sometimes re-sent whole
                close_run(v);
                corro_changeset f = c, s = c;
                f.seq_start = 0;
                f.seq_end = cnt / 2 - 1;
                f.change_count = cnt / 2;
                s.seq_start = cnt / 2;
                s.seq_end = cnt - 1;
                s.change_off = c.change_off + cnt / 2;
                s.change_count = cnt - cnt / 2;
                idx[a].push_back(cs.size());
                cs.push_back(f);
                tail.push_back(cs.size());
                cs.push_back(s);
                if (U(rng) < 0.1) {
                    corro_changeset w = c;
                    w.seq_start = 0;
                    w.seq_end = cnt - 1;
                    w.change_count = cnt;
                    tail.push_back(cs.size());
                    cs.push_back(w);
                }
            } else if (!run0) {
                run0 = v;
            }
        }
        close_run(NV + 1);
        std::shuffle(tail.begin(), tail.end(), rng);
        idx[a].insert(idx[a].end(), tail.begin(), tail.end());
    }
    const uint64_t nh = cs.size();
    std::vector<uint8_t> bad(nh, 0), flag(nh, 0), canon(nh, 1);
    std::vector<int32_t> known(nh, 0);
    std::vector<uint32_t> ctab(nh, 0);
    const CsView view{cs.data(), bad.data(), known.data(), flag.data(), canon.data(), ctab.data()};
    auto row_of = [](const corro_changeset &, uint64_t, uint64_t) -> HostRow { throw std::logic_error("no host rows"); };
    std::vector<double> ms;
    uint64_t spans = 0;
    for (int r = 0; r < reps; r++) {
        corro_bookie *bk = new corro_bookie();
        std::vector<ActorWork> work(NA);
        std::vector<RunView> runs(NA);
        for (uint32_t a = 0; a < NA; a++) {
            ActorWork &w = work[a];
            w.site = a;
            w.id = ids[a];
            w.booked = booked_of_site(bk, a, w.id, true);
            w.had_max = w.booked->has_max;
            w.max = w.booked->max;
            w.idx = idx[a].data();
            w.nidx = idx[a].size();
            runs[a] = RunView{rs[a].data(), re[a].data(), nullptr, rs[a].size()};
        }
        const auto t0 = std::chrono::steady_clock::now();
        if (serial)
            for (uint32_t a = 0; a < NA; a++) run_actor_walk(bk, work[a], view, runs[a], row_of);
        else
            run_parallel(NA, [&](size_t a) { run_actor_walk(bk, work[a], view, runs[a], row_of); });
        ms.push_back(std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count());
        spans = 0;
        for (const ActorWork &w : work) spans += w.nspans;
        delete bk;
    }
    std::sort(ms.begin(), ms.end());
    std::printf("host changesets %llu, walked spans %llu, walk %s: median %.3f ms (min %.3f)\n", (unsigned long long)nh,
                (unsigned long long)spans, serial ? "serial" : "parallel", ms[ms.size() / 2], ms[0]);
    return 0;
}
