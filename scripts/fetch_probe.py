"""Known-bytes probe of the FETCH_SIZE counter (MI355X_MICROARCH.md's x2 correction for gfx950): one launch per load
shape over a fresh 256 MiB buffer, read once. Run under `rocprofv3 --pmc FETCH_SIZE`; the summary divides the counter
by the bytes each launch reads (scripts/fetch_probe_summary.py).

    bash scripts/build_fetch_probe.sh   # variants/libfetch_probe.so (hipcc, gfx950)
"""
import ctypes as C
import json
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def main():
    lib = C.CDLL(os.path.join(ROOT, "variants", "libfetch_probe.so"))
    lib.fetch_probe_run.argtypes = [C.c_int, C.c_void_p, C.c_size_t, C.c_int, C.c_void_p]
    dev = torch.device("cuda", 0)
    nbytes = 256 << 20
    pitch = 1280 + 128   # a 1280-px level's pitch (rounded to 64 B, plus one line)
    sink = torch.zeros(4, dtype=torch.int32, device=dev)
    out = []
    for kind, name in ((0, "wide16"), (1, "dword"), (2, "byte"), (3, "fast_roi")):
        buf = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)   # fresh: not in L2 / MALL from before
        torch.cuda.synchronize()
        flush = torch.empty(512 << 20, dtype=torch.uint8, device=dev).fill_(1)   # evict the buffer from the caches
        torch.cuda.synchronize()
        del flush
        rc = lib.fetch_probe_run(kind, buf.data_ptr(), nbytes, pitch, sink.data_ptr())
        if rc:
            raise RuntimeError("probe launch failed")
        if kind == 3:
            rows = nbytes // pitch
            read = (pitch // 44) * (rows // 41) * 41 * 44
        else:
            read = nbytes
        out.append({"shape": name, "bytes_read": read})
        del buf
    print(json.dumps(out))


if __name__ == "__main__":
    sys.exit(main())
