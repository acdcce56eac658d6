"""Development probe: HIP IPC of a torch device buffer between two processes
on one GPU (the mapping bench.py --gather ipc uses), step by step, with
faulthandler on. usage: python tools/ipc_probe.py"""
import faulthandler
import os
import subprocess
import sys
import time

faulthandler.enable()
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

if len(sys.argv) > 1 and sys.argv[1] == "child":
    import torch
    from bevy_raytrace_amd import distributed as rdist
    torch.cuda.set_device(0)
    torch.zeros(1, device="cuda")
    blob = bytes.fromhex(sys.argv[2])
    print("child: importing", flush=True)
    m, p = rdist.ipc_import(blob)
    print(f"child: mapped {m:#x} ptr {p:#x}", flush=True)
    h = rdist._hip()
    import ctypes
    h.hipMemset.restype = ctypes.c_int
    h.hipMemset.argtypes = [ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t]
    rc = h.hipMemset(ctypes.c_void_p(p), 0x3F, 4096)
    h.hipDeviceSynchronize()
    print(f"child: memset rc={rc}", flush=True)
    rdist.ipc_close(m)
    print("child: closed", flush=True)
    sys.exit(0)

import torch  # noqa: E402
from bevy_raytrace_amd import distributed as rdist  # noqa: E402
torch.cuda.set_device(0)
buf = torch.zeros((4, 1024), dtype=torch.float32, device="cuda")
print(f"parent: ptr {buf.data_ptr():#x}", flush=True)
blob = rdist.ipc_export(buf.data_ptr())
print(f"parent: exported {len(blob)} bytes, offset {int.from_bytes(blob[64:], 'little')}", flush=True)
p = subprocess.run([sys.executable, "-X", "faulthandler", __file__, "child", blob.hex()],
                   capture_output=True, text=True, timeout=120)
print(p.stdout, p.stderr[-3000:], "rc", p.returncode, flush=True)
torch.cuda.synchronize()
v = buf.cpu().view(-1)[:4].numpy()
print("parent: first words after the child's memset:", v, flush=True)
