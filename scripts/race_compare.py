"""Compare two scripts/race_replay.py outputs: which tensors differ (diagnosis helper)."""
import sys

import torch

a = torch.load(sys.argv[1], weights_only=True)
b = torch.load(sys.argv[2], weights_only=True)
diff = [k for k in a if not torch.equal(a[k], b[k])]
print(f"{len(diff)} of {len(a)} differ: {diff[:20]}")
