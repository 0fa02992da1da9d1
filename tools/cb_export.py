#!/usr/bin/env python3
"""Export the cached fitted codebooks (SWEEP_CB npz) compactly (fp32 centres + bit-packed match) so a
GPU run can hand them back through gpurun_out/ for CPU-side analysis."""
import sys
import numpy as np
z = np.load(sys.argv[1])
np.savez(sys.argv[2], c0=z["c0"], c1=z["c1"], c2=z["c2"], match_bits=np.packbits(z["match"].astype(bool), axis=1))
