"""One end of the cross-process HBM sharing check (tests/test_gpu_ipc.py).

export: hipMalloc a buffer on device 0, fill it with seeded random bytes,
        print its hipIpcGetMemHandle (hex), wait for a line on stdin, exit.
import: read a handle (hex) from argv, hipIpcOpenMemHandle it, copy the bytes
        back and compare with the same seeded bytes.
Prints one JSON line: {"role", "ok", "error"}. ctypes against the HIP runtime
PyTorch ships (the one RCCL uses in bench.py), no torch CUDA calls.
"""

import ctypes
import json
import os
import random
import sys

NBYTES = 16 << 20


class Handle(ctypes.Structure):
    _fields_ = [("reserved", ctypes.c_char * 64)]


def hip():
    import torch

    lib = os.path.join(os.path.dirname(torch.__file__), "lib", "libamdhip64.so")
    h = ctypes.CDLL(lib)
    h.hipGetErrorString.restype = ctypes.c_char_p
    return h


def check(h, rc, what):
    if rc != 0:
        raise RuntimeError(f"{what}: {h.hipGetErrorString(rc).decode()} ({rc})")


def payload():
    return random.Random(1234).randbytes(NBYTES)


def main():
    role = sys.argv[1]
    out = {"role": role, "ok": False, "error": "", "legacy_env": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY")}
    try:
        h = hip()
        check(h, h.hipSetDevice(0), "hipSetDevice")
        if role == "export":
            p = ctypes.c_void_p()
            check(h, h.hipMalloc(ctypes.byref(p), ctypes.c_size_t(NBYTES)), "hipMalloc")
            data = payload()
            check(h, h.hipMemcpy(p, data, ctypes.c_size_t(NBYTES), 1), "hipMemcpy H2D")  # hipMemcpyHostToDevice
            hd = Handle()
            check(h, h.hipIpcGetMemHandle(ctypes.byref(hd), p), "hipIpcGetMemHandle")
            print(ctypes.string_at(ctypes.byref(hd), 64).hex(), flush=True)  # (c_char arrays stop at NUL)
            sys.stdin.readline()  # the importer is done
            out["ok"] = True
        else:
            hd = Handle()
            ctypes.memmove(ctypes.byref(hd), bytes.fromhex(sys.argv[2]), 64)
            p = ctypes.c_void_p()
            check(h, h.hipIpcOpenMemHandle(ctypes.byref(p), hd, 1), "hipIpcOpenMemHandle")  # lazy peer access
            buf = ctypes.create_string_buffer(NBYTES)
            check(h, h.hipMemcpy(buf, p, ctypes.c_size_t(NBYTES), 2), "hipMemcpy D2H")  # hipMemcpyDeviceToHost
            out["ok"] = buf.raw == payload()
            if not out["ok"]:
                out["error"] = "bytes differ"
            check(h, h.hipIpcCloseMemHandle(p), "hipIpcCloseMemHandle")
    except Exception as e:  # noqa: BLE001
        out["error"] = str(e)
    print(json.dumps(out), flush=True)
    return 0 if out["ok"] else 1


if __name__ == "__main__":
    sys.exit(main())
