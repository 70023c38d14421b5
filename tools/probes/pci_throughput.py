#!/usr/bin/env python3
"""Is there a directional PCIe byte source on this GPU?  (DCGM fields
1009/1010, pcie_tx_bytes / pcie_rx_bytes, DcgmGroupInfo.cpp:46-47.)

Probes, idle and under a host->device copy load:
  * rsmi_dev_pci_throughput_get (sent / received packets per second and the
    max payload size, from the driver's pcie_bw file)
  * the pcie_bw sysfs file itself
  * gpu_metrics pcie_bandwidth_acc / pcie_bandwidth_inst (total only)
Prints one JSON line."""
import ctypes
import glob
import json
import os
import subprocess
import sys
import time


def smi():
    for p in ("librocm_smi64.so.7", "/opt/rocm/lib/librocm_smi64.so"):
        try:
            lib = ctypes.CDLL(p)
            break
        except OSError:
            lib = None
    if lib is None or lib.rsmi_init(ctypes.c_uint64(0)) != 0:
        return None
    return lib


def throughput(lib, dv):
    s, r, m = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
    t0 = time.time()
    st = lib.rsmi_dev_pci_throughput_get(ctypes.c_uint32(dv), ctypes.byref(s), ctypes.byref(r), ctypes.byref(m))
    return {"status": st, "sent_pkts": s.value, "received_pkts": r.value, "max_pkt_bytes": m.value,
            "call_s": round(time.time() - t0, 3)}


def sysfs_pcie_bw():
    out = {}
    for f in sorted(glob.glob("/sys/class/drm/card*/device/pcie_bw")):
        try:
            out[f] = open(f).read().strip()
        except OSError as e:
            out[f] = f"error: {e}"
    return out


LOAD = r"""
import torch, time
x = torch.empty(256 << 20, dtype=torch.uint8).pin_memory()
y = torch.empty(256 << 20, dtype=torch.uint8, device="cuda")
t0 = time.time(); n = 0
while time.time() - t0 < %f:
    y.copy_(x, non_blocking=True); n += 1
    if n %% 8 == 0: torch.cuda.synchronize()
torch.cuda.synchronize()
print("h2d_gb", n * 0.25 / (time.time() - t0))
"""


def main():
    lib = smi()
    res = {"rsmi": lib is not None, "sysfs_idle": sysfs_pcie_bw()}
    if lib is not None:
        n = ctypes.c_uint32()
        lib.rsmi_num_monitor_devices(ctypes.byref(n))
        res["devices"] = n.value
        res["idle"] = [throughput(lib, d) for d in range(n.value)]
        load = subprocess.Popen([sys.executable, "-c", LOAD % 6.0], stdout=subprocess.PIPE, text=True)
        time.sleep(3.0)
        res["h2d_load"] = [throughput(lib, d) for d in range(n.value)]
        res["sysfs_load"] = sysfs_pcie_bw()
        res["load_out"] = load.communicate(timeout=60)[0].strip()
    print(json.dumps(res))


if __name__ == "__main__":
    main()
