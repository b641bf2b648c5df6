"""CPU-baseline thread probe: the host's cores, the job's cgroup CPU quota, and the
oracle's cfg-2 L-BFGS rate (fp64, N = 60000, 4 iterations) at several OpenMP thread counts."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

O = bench.__graft_entry__.load_oracle()
info = dict(host=bench.host_cpu(), omp_env=os.environ.get("OMP_NUM_THREADS"))
for f in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpuset.cpus.effective", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
    try:
        info[f] = open(f).read().strip()
    except OSError:
        pass
print(json.dumps(info), flush=True)
X, Y = O.synth_mnist(60000, 784, 10)
net = O.Net([784, 128, 10], ["relu", "linear"])
P = net.init_cpu(123)
for t in [int(x) for x in sys.argv[1:]] or [16, 32, 64, 128]:
    O.set_threads(t)
    t0 = time.perf_counter()
    _, rec, inf = net.lbfgs_wolfe(P, X, Y, m=10, max_iters=4)
    dt = time.perf_counter() - t0
    print(json.dumps(dict(threads=t, iters=4, s=round(dt, 3), it_per_s=round(4 / dt, 4), ms=inf["ms"])), flush=True)
