"""C-ABI checks that need no GPU: every symbol include/lkfwd.h declares is
exported by liblkfwd.so, and the ctypes mirror matches the C struct sizes."""
import ctypes as C
import os
import re
import subprocess

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(ROOT, "include", "lkfwd.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(lkf_[a-z_]+)\s*\(", hdr)))


def test_header_declares_entry_points():
    syms = declared_symbols()
    for s in ["lkf_create", "lkf_destroy", "lkf_add_track", "lkf_add_downtrack", "lkf_ctl", "lkf_submit",
              "lkf_submit_device", "lkf_run", "lkf_drain", "lkf_get_state", "lkf_seed_state", "lkf_seq_lookup"]:
        assert s in syms, s


def test_library_exports_every_declared_symbol(pkg):
    lib = os.path.join(ROOT, "livekit-server_amd", "lib", "liblkfwd.so")
    if not os.path.exists(lib):
        subprocess.run(["make", "-s", "-C", os.path.join(ROOT, "livekit-server_amd", "csrc")], check=True)
    out = subprocess.run(["nm", "-D", "--defined-only", lib], capture_output=True, text=True, check=True).stdout
    exported = set(l.split()[-1] for l in out.splitlines() if l.strip())
    missing = [s for s in declared_symbols() if s not in exported]
    assert not missing, missing
    # loads (no compute: no device needed to dlopen)
    C.CDLL(lib)


def test_struct_sizes(abi):
    assert C.sizeof(abi.lkf_pkt) == 64
    assert C.sizeof(abi.lkf_out) == 40
    src = r'''
#include <stdio.h>
#include <stddef.h>
#include "include/lkfwd.h"
int main(void){printf("%zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu %zu\n", sizeof(lkf_tracker_status), sizeof(lkf_alloc_req), sizeof(lkf_allocation), sizeof(lkf_pad_req), sizeof(lkf_cfg), sizeof(lkf_track_params),
 sizeof(lkf_downtrack_params), sizeof(lkf_pkt), sizeof(lkf_out), sizeof(lkf_fwd_state), sizeof(lkf_seq_meta),
 sizeof(lkf_pkt_dd), sizeof(lkf_stream_params), sizeof(lkf_dt_summary), sizeof(lkf_transport_params), sizeof(lkf_video_transition), sizeof(lkf_sender_stats), sizeof(lkf_prov_req), sizeof(lkf_prov_result), sizeof(lkf_alloc_group), sizeof(lkf_dd_tracker_status));return 0;}
'''
    exe = "/tmp/lkf_sizes"
    with open(exe + ".c", "w") as f:
        f.write(src)
    subprocess.run(["gcc", "-I", ROOT, "-o", exe, exe + ".c"], check=True)
    sizes = list(map(int, subprocess.run([exe], capture_output=True, text=True).stdout.split()))
    py = [abi.TRACKER_STATUS_DTYPE.itemsize, abi.ALLOC_REQ_DTYPE.itemsize, abi.ALLOCATION_DTYPE.itemsize, abi.PAD_REQ_DTYPE.itemsize, C.sizeof(abi.lkf_cfg), C.sizeof(abi.lkf_track_params), C.sizeof(abi.lkf_downtrack_params),
          C.sizeof(abi.lkf_pkt), C.sizeof(abi.lkf_out), C.sizeof(abi.lkf_fwd_state), C.sizeof(abi.lkf_seq_meta),
          C.sizeof(abi.lkf_pkt_dd), C.sizeof(abi.lkf_stream_params), abi.DT_SUMMARY_DTYPE.itemsize,
          C.sizeof(abi.lkf_transport_params), abi.VIDEO_TRANSITION_DTYPE.itemsize, abi.SENDER_STATS_DTYPE.itemsize,
          abi.PROV_REQ_DTYPE.itemsize, abi.PROV_RESULT_DTYPE.itemsize, abi.ALLOC_GROUP_DTYPE.itemsize,
          abi.DD_TRACKER_STATUS_DTYPE.itemsize]
    assert sizes == py, (sizes, py)


def test_engine_fails_loudly_without_gpu(pkg):
    import torch
    if torch.cuda.is_available():
        return
    try:
        pkg.Engine(max_downtracks=16, max_tracks=4)
    except pkg.EngineError:
        return
    raise AssertionError("Engine() must raise without a GPU (no CPU fallback)")
