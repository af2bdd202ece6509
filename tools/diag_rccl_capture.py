import os, sys, traceback
sys.path.insert(0, "tests"); sys.path.insert(0, ".")
import torch, torch.distributed as dist
import test_rccl_capture_gpu as t
torch.cuda.set_device(0)
dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{t._free_port()}", rank=0, world_size=1, device_id=torch.device("cuda", 0))
for mode in ("full", "segmented", None):
    try:
        m, out = t._run(mode, "grad", mode is not None, "fp32")
        print("ok", mode, m, flush=True)
    except Exception:
        traceback.print_exc()
        sys.stdout.flush(); sys.stderr.flush()
        os._exit(3)
os._exit(0)
