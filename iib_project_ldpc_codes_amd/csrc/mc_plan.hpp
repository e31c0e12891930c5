// Round accounting of a multi-device Monte-Carlo run (ldpc_mc_run, mc_run.cpp), kept free of
// HIP / RCCL so the host-only debug entry ldpc_debug_mc_plan runs the SAME driver loop on a
// synthetic per-trial frame-error sequence (tests/test_mc_plan.py, on the CPU).
//
// The rule it implements is the reference's sequential loop
//     while frame_errors < stop and trials < num_tests: run one trial
// (parallel_simulator.py:198; expurgated :200), applied to trials that ndev slots decode in
// rounds: slot i of round R decodes trials [(R*ndev + i)*batch, +B_i).
//   * B_i is fixed for the round from the trials counted BEFORE it: the round's batches are
//     clamped, in trial order, so that no trial at or past num_tests runs.
//   * In the round whose frame errors reach `stop`: slots before the crossing keep their
//     whole batch, the crossing slot re-runs the SAME B_i trials with the in-batch cut at its
//     share of the remaining frame errors (the cutoff kernel keeps trials up to and including
//     the one that reaches the quota), later slots drop theirs.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <chrono>
#include <vector>

namespace ldpc {

struct McPlan {
    int64_t num_tests = 0;  // <= 0: no trial limit
    int64_t stop = 0;       // <= 0: no frame-error stop
    int batch = 0, ndev = 1;

    // batch of every slot for a round that starts with `trials_before` trials counted
    std::vector<int> batches(int64_t trials_before) const {
        std::vector<int> B(ndev, batch);
        if (num_tests > 0)
            for (int i = 0; i < ndev; ++i) {
                const int64_t left = num_tests - trials_before - (int64_t)i * batch;
                B[i] = (int)std::max<int64_t>(0, std::min<int64_t>(batch, left));
            }
        return B;
    }
    bool done(int64_t frames, int64_t trials) const {
        return (stop > 0 && frames >= stop) || (num_tests > 0 && trials >= num_tests);
    }
    // the crossing round: action of every slot given the frame errors each found in its
    // whole batch -- 0 keep the whole batch, q > 0 re-run with the cut at q frame errors,
    // -1 drop.  Empty when the round does not reach `stop`.
    std::vector<int64_t> crossing(int64_t frames_before, const std::vector<int64_t> &f) const {
        int64_t sum = 0;
        for (int64_t x : f) sum += x;
        if (stop <= 0 || frames_before + sum < stop) return {};
        std::vector<int64_t> act(ndev, -1);
        int64_t before = frames_before;
        for (int i = 0; i < ndev; ++i) {
            const int64_t quota = stop - before;
            if (quota <= 0) break;
            if (quota > f[i]) {
                act[i] = 0;
                before += f[i];
            } else {
                act[i] = quota;
                break;
            }
        }
        return act;
    }
};

// The driver loop.  Backend:
//   int round(int64_t R, const std::vector<int> &B, std::vector<int64_t> &f)
//        every slot i decodes trials [(R*ndev + i)*batch, +B[i]) into a delta (no cut);
//        the deltas are summed across slots (the all-reduce); f[i] = slot i's frame errors
//   int keep_round()                       counters += the summed delta
//   int keep(int i)                        counters += slot i's delta
//   int cut(int64_t R, int i, int B, int64_t quota)
//        re-run slot i's trials with the in-batch cut at quota; counters += that delta
//   int64_t frames(), trials()             the counters so far
// Returns the first non-zero backend code, else 0; rounds = rounds run.
template <class Backend>
int mc_drive(const McPlan &P, Backend &be, double time_limit_s, int64_t &rounds) {
    const auto t0 = std::chrono::steady_clock::now();
    rounds = 0;
    std::vector<int64_t> f(P.ndev);
    while (!P.done(be.frames(), be.trials())) {
        const std::vector<int> B = P.batches(be.trials());
        const int64_t R = rounds;
        int rc = be.round(R, B, f);
        if (rc) return rc;
        ++rounds;
        const std::vector<int64_t> act = P.crossing(be.frames(), f);
        if (!act.empty()) {
            for (int i = 0; i < P.ndev; ++i) {
                if (act[i] < 0) break;
                rc = act[i] == 0 ? be.keep(i) : be.cut(R, i, B[i], act[i]);
                if (rc) return rc;
            }
            break;
        }
        rc = be.keep_round();
        if (rc) return rc;
        if (time_limit_s > 0 &&
            std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count() > time_limit_s)
            break;
    }
    return 0;
}

}  // namespace ldpc
