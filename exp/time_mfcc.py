import sys, os, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from honk_amd.audio import AudioPreprocessor
ap = AudioPreprocessor()
B = int(sys.argv[1]) if len(sys.argv) > 1 else 16384
x = (torch.rand(B, 16000, device="cuda") * 2 - 1) * 0.3
ap.compute_mfccs_batch(x); torch.cuda.synchronize()
t0 = time.perf_counter()
for _ in range(5): ap.compute_mfccs_batch(x)
torch.cuda.synchronize()
print(f"mfcc {os.environ.get('HONK_MFCC_VALU') and 'valu' or 'mfma'}: {5*B/(time.perf_counter()-t0):.0f} clips/s")
