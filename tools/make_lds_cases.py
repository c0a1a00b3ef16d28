"""Write the messages of tests/test_gpu_inflate.py::test_inflate_lds_table_paths in the
layout tools/prof_infl_tok.hip reads (to count the LDS path's HBM-table fallbacks)."""
import sys
import zlib

import numpy as np

sys.path.insert(0, ".")
from snf4j_amd._lib import DESC_DTYPE  # noqa: E402
from tests.test_gpu_inflate import _lds_path_messages  # noqa: E402

kinds = _lds_path_messages(np.random.default_rng(0x1D5))
comp = [(c.compress(b) + c.flush(zlib.Z_SYNC_FLUSH))[:-4] for _, b, c in kinds]
n = len(comp)
desc = np.zeros(n, dtype=DESC_DTYPE)
off = np.zeros(n + 1, dtype=np.uint64)
np.cumsum([len(x) for x in comp], out=off[1:])
desc["payload_off"], desc["payload_len"], desc["opcode"], desc["flags"] = off[:-1], [len(x) for x in comp], 1, 0xC0
payload = np.frombuffer(b"".join(comp) + bytes(16), dtype=np.uint8)
with open(sys.argv[1], "wb") as f:
    f.write(np.array([n, n, payload.size, 65536], dtype=np.uint64).tobytes())
    f.write(desc.tobytes())
    f.write(np.arange(n + 1, dtype=np.uint32).tobytes())
    f.write(payload.tobytes())
