"""The GPU box's host CPUs as this process sees them (affinity, machine count, the harness's
thread share) — what bench.py's CPU baseline sizes its threads by."""
import os
import platform

aff = sorted(os.sched_getaffinity(0))
print(f"affinity {len(aff)} cpus (first {aff[:4]} last {aff[-2:]}); os.cpu_count {os.cpu_count()}; "
      f"OMP_NUM_THREADS {os.environ.get('OMP_NUM_THREADS')}; machine {platform.machine()}")
try:
    model = [line.split(":", 1)[1].strip() for line in open("/proc/cpuinfo") if line.startswith("model name")]
    print(f"cpu model {model[0] if model else '?'}")
except OSError:
    pass
