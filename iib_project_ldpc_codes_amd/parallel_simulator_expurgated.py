"""Mirror of parallel_simulator_expurgated.py: a trial counts only if its residual
erasure count exceeds ``expurgation`` (argv[9]; parallel_simulator_expurgated.py:238-243),
CSV names prefixed ``regular_code_expurgated=<X>`` (:262-263)."""
import sys

from . import parallel_simulator as ps
from .parallel_simulator import regular_LDPC_code  # noqa: F401  (same class as the reference)


def run_simulation(parameter_set):
    X = int(parameter_set["expurgation"])
    return ps._run(parameter_set, fixed=False, expurgation=X, prefix="regular_code_expurgated=" + str(X),
                   time_limit=float("inf"))


def run_simulation_fixed_ldpc(parameter_set):
    X = int(parameter_set.get("expurgation", -1))
    return ps._run(parameter_set, fixed=True, expurgation=X, prefix="regular_code_expurgated=" + str(X),
                   time_limit=42000.0)


def main(argv=None):
    """eps num_tests iterations n dv dc mode seed|filenumber expurgation (:416-459)."""
    argv = sys.argv[1:] if argv is None else argv
    erasure_prob = float(argv[0])
    num_tests, iterations, n, dv, dc, mode = (int(a) for a in argv[1:7])
    expurgation = int(argv[8])
    if mode not in range(6):
        raise ValueError("Mode value must be in the range 0-5")
    base = {"BEC": erasure_prob, "num_tests": num_tests, "iterations": iterations, "n": n, "dv": dv, "dc": dc,
            "optimal": mode in (1, 2, 4, 5), "message_passing": mode in (0, 2, 3, 5)}
    if mode < 3:
        return run_simulation(dict(base, expurgation=expurgation, seed=int(argv[7])))
    return run_simulation_fixed_ldpc(dict(base, expurgation=expurgation, filenumber=int(argv[7])))


if __name__ == "__main__":
    main()
