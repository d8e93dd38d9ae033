"""Print this process's allowed CPUs, their NUMA nodes, and the GPU's NUMA node (sysfs; no GPU call).
`--local` prints the allowed CPUs on the GPU's NUMA node as a taskset list (all allowed CPUs if none)."""
import glob, os, sys

def cpu_node(c):
    for p in glob.glob(f"/sys/devices/system/cpu/cpu{c}/node*"):
        return int(p.rsplit("node", 1)[1])
    return -1

def gpu_nodes():
    out = []
    for d in sorted(glob.glob("/sys/class/drm/card*/device")):
        try:
            vendor = open(d + "/vendor").read().strip()
            node = int(open(d + "/numa_node").read().strip())
        except OSError:
            continue
        if vendor == "0x1002" and os.path.exists(d + "/numa_node"):
            out.append((os.path.realpath(d).rsplit("/", 1)[1], node))
    return out

cpus = sorted(os.sched_getaffinity(0))
g = gpu_nodes()
if "--local" in sys.argv:
    nodes = {n for _, n in g}
    loc = [c for c in cpus if cpu_node(c) in nodes] or cpus
    print(",".join(map(str, loc)))
else:
    print("allowed cpus:", cpus)
    print("cpu nodes:", sorted({(cpu_node(c)) for c in cpus}), [(c, cpu_node(c)) for c in cpus])
    print("gpus (pci, numa):", g)
    print("HIP_VISIBLE_DEVICES", os.environ.get("HIP_VISIBLE_DEVICES"), "ROCR_VISIBLE_DEVICES", os.environ.get("ROCR_VISIBLE_DEVICES"))
