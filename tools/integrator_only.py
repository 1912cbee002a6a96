"""The bench's integrator HBM-roofline leg alone (2^20 rays x 128 samples, render fwd + bwd), for
rocprofv3 passes that must not mix in the training step's small render launches."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import bench  # noqa: E402

import torch  # noqa: E402

import nof  # noqa: E402

print(json.dumps(bench.integrator_roofline(torch, nof, torch.device("cuda", 0))), flush=True)
