"""Phase timeline of the host reduce->bcast myAllreduce (CCMPI_P2P_TRACE=1): per run, every
rank's barrier exit and the schedule's phase marks on one monotonic clock, relative to the
earliest barrier exit; rank 0 prints the mean timeline per rank for fresh / reused arrays."""
import json
import os
import sys

os.environ.setdefault("CCMPI_P2P_TRACE", "1")  # 2: also the marks inside isend_raw
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import numpy as np  # noqa: E402

from collective_communication_mpi_amd import MPI, Communicator, _native  # noqa: E402

if os.environ.get("HT_PIN"):  # pin rank r to CPU HT_PIN + r (one L3 domain for 8 ranks)
    os.sched_setaffinity(0, {int(os.environ["HT_PIN"]) + int(os.environ.get("RANK", os.environ.get("CCMPI_RANK", "0")))})
if os.environ.get("HT_GC") == "0":  # diagnostic: no cyclic-GC passes during the loop
    import gc
    gc.disable()
world = MPI.COMM_WORLD
comm = Communicator(world)
rank, p = comm.Get_rank(), comm.Get_size()
rng = np.random.default_rng(rank)
n, runs = 1024, 200
H = _native.host()
src0 = rng.standard_normal(n).astype(np.float32)
keep = []  # fresh_nofree: every run's arrays stay alive (new addresses and pages every run)
for fresh in os.environ.get("HT_MODES", "fresh,reuse").split(","):
    s = rng.standard_normal(n).astype(np.float32)
    d = np.empty(n, np.float32)
    rows = []
    H.p2p_trace()
    for _ in range(runs):
        if fresh == "fresh":      # the reference's loop: new random source, new result array
            s = rng.standard_normal(n).astype(np.float32)
            d = np.empty(n, np.float32)
        elif fresh == "rngwork":  # the same random-number work, arrays reused
            rng.standard_normal(n).astype(np.float32)
        elif fresh == "copyfresh":  # new arrays without the random-number work
            s = src0.copy()
            d = np.empty(n, np.float32)
        elif fresh == "fresh_nofree":  # nothing freed: every run on never-touched heap memory
            s = rng.standard_normal(n).astype(np.float32)
            d = np.empty(n, np.float32)
            keep.append((s, d))
        elif fresh == "fresh_touch_s":  # the reference's loop + the source re-read before the barrier
            s = rng.standard_normal(n).astype(np.float32)
            d = np.empty(n, np.float32)
            float(s.sum())
        elif fresh == "fresh_touch_d":  # the reference's loop + the result written before the barrier
            s = rng.standard_normal(n).astype(np.float32)
            d = np.empty(n, np.float32)
            d.fill(0)
        elif fresh == "pool":  # 64 pre-touched (source, result) pairs in turn: new addresses, warm pages
            if not hasattr(sys, "_ht_pool"):
                sys._ht_pool = [(rng.standard_normal(n).astype(np.float32), np.zeros(n, np.float32)) for _ in range(64)]
                sys._ht_i = 0
            s, d = sys._ht_pool[sys._ht_i % 64]
            sys._ht_i += 1
        comm.Barrier()
        t0 = H.wtime()
        comm.myAllreduce(s, d, op=MPI.MIN)
        t1 = H.wtime()
        comm.Barrier()
        rows.append([t0] + H.p2p_trace() + [t1])
    allrows = world.gather(rows, root=0)
    if rank == 0:
        out = {}
        for r in range(p):
            rel = []
            for k in range(runs):
                t_first = min(allrows[q][k][0] for q in range(p))
                rel.append([x - t_first for x in allrows[r][k]])
            m = np.mean(np.array(rel[20:]), axis=0) * 1e6
            out[r] = [round(float(x), 2) for x in m]
        print(json.dumps({"fresh": fresh, "timeline_us": out}), flush=True)
