import sys, time
sys.path.insert(0, 'nerf-or-nothing_amd')
import nof
from nof.dp import NativeDP
t0 = time.time()
print("start", flush=True)
try:
    NativeDP.init_rank(NativeDP.unique_id(), 2, 0, 0, timeout_ms=3000)
    print("NO-ERROR", flush=True)
except nof.NofError as e:
    print("STATUS", e.status, round(time.time() - t0, 1), e, flush=True)
