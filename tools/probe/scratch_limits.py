"""Print the HSA runtime's scratch limits and the KFD topology fields that size a queue's scratch reservation
(HSA_AMD_AGENT_INFO_SCRATCH_LIMIT_MAX / _CURRENT, hsa_ext_amd.h:686-703; max_slots_scratch_cu from the KFD topology).
Diagnostic only: no kernel is launched."""
import ctypes, glob, json, os

hsa = ctypes.CDLL("/opt/rocm/lib/libhsa-runtime64.so")
assert hsa.hsa_init() == 0
agents = []
CB = ctypes.CFUNCTYPE(ctypes.c_int, ctypes.c_uint64, ctypes.c_void_p)


def cb(agent, _):
    t = ctypes.c_uint32()
    hsa.hsa_agent_get_info(ctypes.c_uint64(agent), 17, ctypes.byref(t))   # HSA_AGENT_INFO_DEVICE
    if t.value == 1:                                                       # HSA_DEVICE_TYPE_GPU
        agents.append(agent)
    return 0


hsa.hsa_iterate_agents(CB(cb), None)
out = []
for a in agents:
    rec = {}
    for name, attr, ty in [("scratch_limit_max", 0xA116, ctypes.c_uint64), ("scratch_limit_current", 0xA117, ctypes.c_uint64),
                           ("cu_count", 0xA002, ctypes.c_uint32), ("max_waves_per_cu", 0xA00A, ctypes.c_uint32),
                           ("simds_per_cu", 0xA00B, ctypes.c_uint32), ("num_xcc", 0xA111, ctypes.c_uint32)]:
        v = ty()
        rc = hsa.hsa_agent_get_info(ctypes.c_uint64(a), attr, ctypes.byref(v))
        rec[name] = v.value if rc == 0 else f"rc={rc:#x}"
    out.append(rec)
print(json.dumps(out))
for p in sorted(glob.glob("/sys/class/kfd/kfd/topology/nodes/*/properties")):
    try:
        kv = dict(l.split()[:2] for l in open(p) if l.strip())
    except OSError as e:                  # (not readable by the box's user)
        print(p, "unreadable:", e)
        continue
    if int(kv.get("simd_count", 0)) > 0:
        print(p, {k: kv[k] for k in kv if "scratch" in k or k in ("simd_count", "num_xcc", "max_waves_per_simd",
                                                               "cu_per_simd_array", "simd_per_cu", "array_count")})
for k in ("GPU_MAX_HW_QUEUES", "HSA_SCRATCH_SINGLE_LIMIT", "HSA_SCRATCH_SINGLE_LIMIT_ASYNC", "HSA_SCRATCH_MEM",
          "HSA_ENABLE_SCRATCH_ASYNC_RECLAIM", "HSA_NO_SCRATCH_RECLAIM"):
    print(k, os.environ.get(k))
