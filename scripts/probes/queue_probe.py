"""Which hardware queue does each HIP stream land on?  Run under rocprofv3 --kernel-trace:
every stream launches one tagged fill (a distinct element count per stream), and the trace's
Queue_Id column of each launch names the queue.  Env GPU_MAX_HW_QUEUES as given."""
import os
import sys

import torch

n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
dev = torch.device("cuda:0")
streams = [torch.cuda.Stream(dev) for _ in range(n)]
hi = [torch.cuda.Stream(dev, priority=-1) for _ in range(2)]
bufs = []
for i, s in enumerate(streams + hi):
    with torch.cuda.stream(s):
        b = torch.empty(1000 + i, device=dev)
        b.fill_(float(i))  # grid size tags the stream
        bufs.append(b)
torch.cuda.synchronize()
print("streams", [hex(s.cuda_stream) for s in streams + hi], "GPU_MAX_HW_QUEUES",
      os.environ.get("GPU_MAX_HW_QUEUES"))
