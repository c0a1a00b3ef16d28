"""Write the bench's permessage-deflate batch (snf4j_amd.synth.deflate_batch) in the
binary layout tools/prof_inflate.hip reads."""
import sys

import numpy as np

sys.path.insert(0, ".")
from benchsupport.synth import deflate_batch  # noqa: E402

n_s = int(sys.argv[2]) if len(sys.argv) > 2 else 1024
desc, sf, payload, plain = deflate_batch(0x1F1A, n_s, 16, 4096)
with open(sys.argv[1] if len(sys.argv) > 1 else "gpurun_out/infl_in.bin", "wb") as f:
    f.write(np.array([len(desc), n_s, payload.size, 16 * 4096], dtype=np.uint64).tobytes())
    f.write(desc.tobytes())
    f.write(sf.astype(np.uint32).tobytes())
    f.write(payload.tobytes())
