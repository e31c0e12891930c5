"""One-node multi-GPU launch for the host-side drivers (bench.py, scripts/fer_sweep.py): one
process per GPU, decided before anything initialises HIP, started as child processes (never
exec), refused when more ranks are asked for than GPUs are visible.  The reference fans its
Monte-Carlo out as independent processes (parallel_simulator.py:403-445); here the ranks share
one torch.distributed group and all-reduce their counters (montecarlo.py)."""
import os
import sys
import time


def launch_plan(gpus, env, visible, rehearse=False):
    """How this invocation runs, decided BEFORE anything initialises HIP:
      ("single", None)  one process, one GPU (--gpus 1, no WORLD_SIZE)
      ("rank", None)    a rank of an external launcher (torchrun: WORLD_SIZE == --gpus)
      ("spawn", envs)   bench.py starts --gpus ranks itself, one child process per GPU, with
                        these environments (RANK / LOCAL_RANK / WORLD_SIZE / MASTER_*)
      ("error", msg)    refused (never a 1-GPU line for --gpus N)
    visible = GPUs this process can see (torch.cuda.device_count(), which does not
    initialise the runtime on this image)."""
    if gpus < 1:
        return "error", f"--gpus {gpus}: need at least one GPU"
    world = env.get("WORLD_SIZE")
    if world is not None:
        if int(world) != gpus:
            return "error", f"--gpus {gpus} but the launcher started WORLD_SIZE={world} ranks"
        if not rehearse and gpus > visible:
            return "error", f"--gpus {gpus} but only {visible} GPU(s) visible"
        return "rank", None
    if gpus > visible and not rehearse:
        return "error", (f"--gpus {gpus} but only {visible} GPU(s) visible to this process "
                         f"(use --rehearse-on-one-gpu to rehearse the {gpus}-rank path on fewer devices)")
    if gpus == 1:
        return "single", None
    port = env.get("MASTER_PORT") or str(_free_port())
    envs = []
    for r in range(gpus):
        e = dict(env)
        e.update({"RANK": str(r), "LOCAL_RANK": str(r), "WORLD_SIZE": str(gpus), "LOCAL_WORLD_SIZE": str(gpus),
                  "MASTER_ADDR": "127.0.0.1", "MASTER_PORT": port})
        if rehearse:
            e["LDPC_DIST_BACKEND"] = "gloo"  # ranks share a device: RCCL needs one rank per GPU
        envs.append(e)
    return "spawn", envs


def _free_port():
    import socket
    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as sk:
        sk.bind(("127.0.0.1", 0))
        return sk.getsockname()[1]


class _Stop(Exception):
    def __init__(self, signum):
        super().__init__(signum)
        self.signum = signum


def spawn_ranks(envs, argv, script=None, grace=5.0):
    """Start one child process per rank (never exec: this process has not touched the GPU,
    and stays the parent); rank 0's stdout (the JSON line) passes through.  Returns the
    worst exit code; if a rank fails the others are terminated.  SIGTERM / SIGHUP / SIGINT
    aimed at this process alone (a scheduler or watchdog that signals only the parent) are
    forwarded: the ranks get SIGTERM, then SIGKILL after `grace` seconds, and the parent
    returns 128 + signum -- no rank is left holding a GPU or writing checkpoints."""
    import signal
    import subprocess
    script = script or os.path.abspath(sys.argv[0])

    def _raise(signum, _frame):
        raise _Stop(signum)

    saved = {}
    for sig in (signal.SIGTERM, signal.SIGHUP, signal.SIGINT):
        try:
            saved[sig] = signal.signal(sig, _raise)
        except ValueError:  # not the main thread: no handlers (the finally block still reaps)
            pass
    procs = []
    rc = 0
    try:
        for e in envs:  # appended one by one: a signal mid-spawn still reaps the ranks already started
            procs.append(subprocess.Popen([sys.executable, "-u", script] + list(argv), env=e))
        while procs:
            for p in list(procs):
                c = p.poll()
                if c is None:
                    continue
                procs.remove(p)
                if c != 0:
                    rc = rc or c
                    for q in procs:  # a failed rank: the others would wait in a collective forever
                        q.terminate()
            time.sleep(0.05)
    except _Stop as st:
        rc = 128 + st.signum
    finally:
        for sig, h in saved.items():
            signal.signal(sig, h)
        for p in procs:
            if p.poll() is None:
                p.terminate()
        t_end = time.time() + grace
        for p in procs:
            try:
                p.wait(timeout=max(0.0, t_end - time.time()))
            except subprocess.TimeoutExpired:
                p.kill()
                p.wait()
    return rc
