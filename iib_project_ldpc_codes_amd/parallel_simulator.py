"""Mirror of the reference's simulator surface (parallel_simulator.py), MI355X-backed.

Same names, argument meaning and output format as the reference:
  * ``regular_LDPC_code(parity_check, n, k, dv, dc).message_pass_decode(binary_sequence,
    max_its, check_lookup=None, variable_lookup=None)`` -> ``(word_int32, errors)`` with
    the initial erasure count prepended (parallel_simulator.py:131-166), calling the
    drop-in ``message_passing`` symbol of libldpc_mi355x.so through ctypes;
  * ``run_simulation`` / ``run_simulation_fixed_ldpc`` (parallel_simulator.py:168-401)
    with the same parameter_set dict keys, stop rules, CSV rows and file names;
  * ``main(argv)``: ``eps num_tests iterations n dv dc mode seed|filenumber``
    (parallel_simulator.py:403-445).

Engines: ``engine="device"`` (default) runs the trial loop as fused device
batches (montecarlo.MonteCarlo: Philox channel, exact sequential stop rule);
``engine="per_trial"`` keeps the reference's per-trial loop (numpy channel,
one drop-in call per trial).  ML ("optimal") decoding (modes 1, 2, 4, 5) runs
on the device too: ``optimal_decode`` calls ldpc_ml_decode_batch, the device
engine ldpc_mc_ml_batch_dev.
"""
import csv
import ctypes as ct
import os
import sys
from datetime import datetime

import numpy as np

from . import _native
from .channels import BEC
from .graph import TannerGraph

base_directory = os.environ.get("LDPC_BASE_DIRECTORY", os.getcwd() + os.sep)
DEFAULT_BATCH = 4096


def _out_path(filename):
    d = os.path.join(base_directory, "report_data", "simulation_data")
    os.makedirs(d, exist_ok=True)
    return os.path.join(d, filename)


def write_optimal_file(filename, optimal_block_error, optimal_bit_error):
    with open(_out_path(filename), "w", newline="") as csvfile:
        writer = csv.writer(csvfile)
        writer.writerow(["Optimal decoding block-wise error", optimal_block_error])
        writer.writerow(["Optimal decoding bit-wise error", optimal_bit_error])


def write_message_passing_file(filename, errors, message_passing_block_error, message_passing_bit_error):
    with open(_out_path(filename), "w", newline="") as csvfile:
        writer = csv.writer(csvfile)
        for error_at_iteration in errors:
            writer.writerow([error_at_iteration])
        writer.writerow(["Message passing block-wise error", message_passing_block_error])
        writer.writerow(["Message passing bit-wise error", message_passing_bit_error])


def write_combined_file(filename, errors, message_passing_block_error, message_passing_bit_error,
                        optimal_block_error, optimal_bit_error):
    with open(_out_path(filename), "w", newline="") as csvfile:
        writer = csv.writer(csvfile)
        for error_at_iteration in errors:
            writer.writerow([error_at_iteration])
        writer.writerow(["Message passing block-wise error", message_passing_block_error])
        writer.writerow(["Message passing bit-wise error", message_passing_bit_error])
        writer.writerow(["Optimal decoding block-wise error", optimal_block_error])
        writer.writerow(["Optimal decoding bit-wise error", optimal_bit_error])


class regular_LDPC_code:  # noqa: N801  (reference name)
    def __init__(self, parity_check, n, k, dv, dc):
        self.parity_check = parity_check
        self.n = n
        self.k = k
        self.dv = dv
        self.dc = dc
        self.rate = self.k / self.n

    def _graph(self):
        if getattr(self, "_tanner", None) is None:
            self._tanner = TannerGraph.from_parity_check(np.asarray(self.parity_check))
        return self._tanner

    def optimal_decode(self, binary_sequence):
        """parallel_simulator.py:60-129 on libldpc_mi355x.so (ldpc_ml_decode_batch):
        erasures (2) solved by GF(2) elimination, 2 left where the reference's loop
        gives an unknown up; words with no erasure or more than n-k are returned as given."""
        from .decoder import ml_decode
        word = np.asarray(binary_sequence)
        no_erasures = np.count_nonzero(word == 2)
        if no_erasures == 0 or no_erasures > (self.n - self.k):
            print("Either no erasures, or too many to be able to solve")
            return binary_sequence
        out, _ = ml_decode(self._graph(), word.astype(np.uint8)[None, :])
        return out[0].astype(np.int64)

    def message_pass_decode(self, binary_sequence, max_its, check_lookup=None, variable_lookup=None):
        """parallel_simulator.py:131-166, backed by libldpc_mi355x.so:message_passing."""
        if check_lookup is None:
            check_lookup = [list(np.nonzero(row == 1)[0]) for row in self.parity_check]
        if variable_lookup is None:
            variable_lookup = [list(np.nonzero(col == 1)[0]) for col in self.parity_check.T]
        check_lookup = np.array(check_lookup, dtype="int32").flatten()
        variable_lookup = np.array(variable_lookup, dtype="int32").flatten()
        errors = np.zeros(max_its, dtype="int32")
        initial_error_count = len(np.nonzero(binary_sequence == 2)[0])
        binary_sequence = np.array(binary_sequence, dtype="int32")
        it = _native.lib().message_passing(binary_sequence.ctypes.data, ct.c_int(max_its),
                                           variable_lookup.ctypes.data, check_lookup.ctypes.data,
                                           errors.ctypes.data, ct.c_int(self.n), ct.c_int(self.k),
                                           ct.c_int(self.dv), ct.c_int(self.dc))
        _native.check(it, "message_passing")
        self.last_it = it
        errors = np.insert(errors, 0, initial_error_count)
        return binary_sequence, errors


def _filename(prefix, parameter_set, n, k, dv, dc, iterations, num, code_number=None, message_passing=True):
    filename = prefix
    if code_number is not None:
        filename += "_code_number=" + str(code_number)
    filename += "_BEC=" + str(parameter_set["BEC"])
    filename += "_n=" + str(n) + "_k=" + str(k) + "_dv=" + str(dv) + "_dc=" + str(dc)
    if message_passing:
        filename += "_it=" + str(iterations)
    filename += "_num=" + str(num)
    filename += "_time=" + datetime.now().strftime("%d-%m-%Y-%H-%M-%S")
    return filename + ".csv"


def _device_loop(graph_fn, parameter_set, expurgation, stop_frames, time_limit):
    """Fused device trial loop; graph_fn(i) gives the graph for batch i (fixed code:
    always the same; ensemble: a fresh draw per ``trials_per_code`` trials)."""
    from .montecarlo import MonteCarlo
    num_tests = parameter_set["num_tests"]
    iterations = parameter_set["iterations"]
    batch = int(parameter_set.get("batch", DEFAULT_BATCH))
    seed = int(parameter_set.get("seed", parameter_set.get("filenumber", 0)))
    per_code = int(parameter_set.get("trials_per_code", 0))  # 0: one fixed code
    t0 = datetime.now()
    counters, res, done, i = None, None, 0, 0
    while done < num_tests:
        B = min(batch if per_code == 0 else per_code, num_tests - done)
        mc = MonteCarlo(graph_fn(i), "bec", parameter_set["BEC"], iterations, expurgation=expurgation,
                        seed=seed, batch=B)
        if counters is not None:
            mc.counters.copy_(counters)
        mc.run_batch(done, B, stop_frames)  # trial indices continue across batches
        counters = mc.counters
        res = mc.results()
        done = res["num_tests"]
        i += 1
        if res["frame_errors"] >= stop_frames:
            break
        if time_limit and (datetime.now() - t0).total_seconds() >= time_limit:
            break
    return res


def _device_ensemble_loop(parameter_set, expurgation, stop_frames, time_limit):
    """Ensemble mode on the device: trial t draws its own code (ldpc_sample_regular law)
    and channel word, decoded and counted in fused batches."""
    from .montecarlo import MonteCarlo
    n, dv, dc = parameter_set["n"], parameter_set["dv"], parameter_set["dc"]
    mc = MonteCarlo.ensemble(n, dv, dc, "bec", parameter_set["BEC"], parameter_set["iterations"],
                             expurgation=expurgation, seed=int(parameter_set.get("seed", 0)),
                             batch=int(parameter_set.get("batch", 1024)))
    t0 = datetime.now()
    num_tests = parameter_set["num_tests"]
    while True:
        done = int(mc.counters[0].item())
        B = min(mc.batch, num_tests - done)
        if B <= 0:
            break
        mc.run_batch(done, B, stop_frames)
        res = mc.results()
        if res["frame_errors"] >= stop_frames or res["num_tests"] >= num_tests:
            break
        if time_limit and (datetime.now() - t0).total_seconds() >= time_limit:
            break
    return mc.results()


def _per_trial_loop(LDPC_fn, parameter_set, expurgation, stop_frames, time_limit, optimal=False,
                    message_passing=True):
    """The reference's own loop (parallel_simulator.py:198-244) with per-trial drop-in calls."""
    sim_BEC = BEC(parameter_set["BEC"])
    num_tests = parameter_set["num_tests"]
    iterations = parameter_set["iterations"]
    n = parameter_set["n"]
    curve = np.zeros(iterations + 1)
    frames = bits = ml_frames = ml_bits = 0
    i = 0
    start = datetime.now()
    while ((frames if message_passing else ml_frames) < stop_frames and i < num_tests
           and (datetime.now() - start).total_seconds() < time_limit):
        LDPC, check_lookup, variable_lookup = LDPC_fn(i)
        channel_output = sim_BEC.new_transmit(np.zeros(n))
        if message_passing:
            _, errors = LDPC.message_pass_decode(channel_output, iterations, check_lookup, variable_lookup)
            if errors[-1] > expurgation:
                curve += errors
                if errors[-1] != 0:
                    frames += 1
                bits += errors[-1]
        if optimal:
            decoded = LDPC.optimal_decode(channel_output)
            count = int(np.count_nonzero(np.asarray(decoded) == 2))
            ml_frames += count > 0
            ml_bits += count
        i += 1
    return {"num_tests": i, "frame_errors": frames, "bit_errors": int(bits),
            "error_curve": curve / (n * i) if i else curve, "ml_frame_errors": int(ml_frames),
            "ml_bit_errors": int(ml_bits)}


def _device_ml_loop(graph, parameter_set, expurgation, stop_frames, time_limit):
    """Optimal modes on the device: ML (+ message passing) per trial in fused batches."""
    from .montecarlo import MonteCarlo
    mp = bool(parameter_set.get("message_passing", True))
    mc = MonteCarlo(graph, "bec", parameter_set["BEC"], parameter_set["iterations"], expurgation=expurgation,
                    seed=int(parameter_set.get("seed", parameter_set.get("filenumber", 0))),
                    batch=int(parameter_set.get("batch", DEFAULT_BATCH)), optimal=True, message_passing=mp)
    t0 = datetime.now()
    num_tests = parameter_set["num_tests"]
    while True:
        res = mc.results()
        done = res["num_tests"]
        B = min(mc.batch, num_tests - done)
        if B <= 0:
            break
        mc.run_batch(done, B, stop_frames)
        res = mc.results()
        frames = res["frame_errors"] if mp else res["ml_frame_errors"]
        if frames >= stop_frames or res["num_tests"] >= num_tests:
            break
        if time_limit and (datetime.now() - t0).total_seconds() >= time_limit:
            break
    return mc.results()


def _run(parameter_set, fixed, expurgation=-1, prefix="regular_code", time_limit=43000.0):
    n, dv, dc = parameter_set["n"], parameter_set["dv"], parameter_set["dc"]
    iterations = parameter_set["iterations"]
    k = int(n * (dc - dv) / dc)
    optimal = bool(parameter_set.get("optimal"))
    message_passing = bool(parameter_set.get("message_passing", True))
    engine = parameter_set.get("engine", "device")
    seed = int(parameter_set.get("seed", parameter_set.get("filenumber", 0)))
    if fixed:
        code = load_or_create_fixed_code(parameter_set["filenumber"], n, dv, dc)
        fn_graph = lambda i: code  # noqa: E731
    else:
        fn_graph = lambda i: TannerGraph.random_regular(n, dv, dc, seed=(seed, i))  # noqa: E731
    if engine == "device" and optimal:
        from .montecarlo import _Ensemble
        res = _device_ml_loop(code if fixed else _Ensemble(n, dv, dc), parameter_set, expurgation, 200, time_limit)
    elif engine == "device" and not fixed:
        res = _device_ensemble_loop(parameter_set, expurgation, 200, time_limit)
    elif engine == "device":
        res = _device_loop(fn_graph, parameter_set, expurgation, 200, time_limit)
    else:
        def ldpc_fn(i):
            g = fn_graph(i)
            return (regular_LDPC_code(g.parity_check(), n, k, dv, dc), g.check_lookup, g.variable_lookup)
        res = _per_trial_loop(ldpc_fn, parameter_set, expurgation, 200, time_limit, optimal, message_passing)
    num_tests = res["num_tests"]
    fname = _filename(prefix, parameter_set, n, k, dv, dc, iterations, num_tests,
                      code_number=parameter_set["filenumber"] if fixed else None, message_passing=message_passing)
    if parameter_set.get("write_csv", True):
        if optimal and message_passing:
            write_combined_file(fname, res["error_curve"], res["frame_errors"] / num_tests,
                                res["bit_errors"] / (num_tests * n), res["ml_frame_errors"] / num_tests,
                                res["ml_bit_errors"] / (num_tests * n))
        elif optimal:
            write_optimal_file(fname, res["ml_frame_errors"] / num_tests, res["ml_bit_errors"] / (num_tests * n))
        else:
            write_message_passing_file(fname, res["error_curve"], res["frame_errors"] / num_tests,
                                       res["bit_errors"] / (num_tests * n))
    res["filename"] = fname
    return res


def load_or_create_fixed_code(filenumber, n, dv, dc):
    """parallel_simulator.py:289-335: reuse parity_checks/{code,check,variable}_code_no_* .npy
    files when present, else draw a code and save them."""
    d = os.path.join(base_directory, "parity_checks")
    os.makedirs(d, exist_ok=True)
    tag = "code_no_" + str(filenumber) + "_n_" + str(n) + "_dv_" + str(dv) + "_dc_" + str(dc) + ".npy"
    paths = [os.path.join(d, tag), os.path.join(d, "check_" + tag), os.path.join(d, "variable_" + tag)]
    k = int(n * (dc - dv) / dc)
    if all(os.path.exists(p) for p in paths[1:]):
        check_lookup = np.load(paths[1], allow_pickle=False)
        variable_lookup = np.load(paths[2], allow_pickle=False)
        return TannerGraph(variable_lookup, check_lookup, n, k, dv, dc)
    g = TannerGraph.random_regular(n, dv, dc, seed=int(filenumber))
    np.save(paths[0], g.parity_check().astype(bool))
    np.save(paths[1], g.check_lookup)
    np.save(paths[2], g.variable_lookup)
    return g


def run_simulation(parameter_set):
    """Ensemble (fresh code per trial): parallel_simulator.py:168-272."""
    return _run(parameter_set, fixed=False)


def run_simulation_fixed_ldpc(parameter_set):
    """Fixed code (concentration plots): parallel_simulator.py:274-401."""
    return _run(parameter_set, fixed=True, time_limit=42000.0)


def main(argv=None):
    """CLI of parallel_simulator.py:403-445: eps num_tests iterations n dv dc mode seed|filenumber."""
    argv = sys.argv[1:] if argv is None else argv
    erasure_prob = float(argv[0])
    num_tests, iterations, n, dv, dc, mode = (int(a) for a in argv[1:7])
    base = {"BEC": erasure_prob, "num_tests": num_tests, "iterations": iterations, "n": n, "dv": dv, "dc": dc}
    if mode not in range(6):
        raise ValueError("Mode value must be in the range 0-5")
    optimal = mode in (1, 2, 4, 5)
    message_passing = mode in (0, 2, 3, 5)
    key = "seed" if mode < 3 else "filenumber"
    ps = dict(base, optimal=optimal, message_passing=message_passing, **{key: int(argv[7])})
    return run_simulation(ps) if mode < 3 else run_simulation_fixed_ldpc(ps)


if __name__ == "__main__":
    main()
