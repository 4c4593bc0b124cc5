"""Square / long-K GEMM shapes for the large-tile variants (diagnostic)."""
import sys
sys.path.insert(0, __import__("os").path.dirname(__file__))
import gemm_bench as gb  # noqa: E402
from dsvt import _lib  # noqa: E402

shapes = [(4096, 4096, 4096), (8192, 8192, 8192), (25104, 2304, 768), (25088, 2304, 3072), (25088, 2048, 768)]
vs = [int(v) for v in sys.argv[1:]] or [10, 20]
for M, N, K in shapes:
    tf, ms = gb.torch_ref(M, N, K)
    cells = ["blas %.0f" % tf]
    for v in vs:
        best = 0
        for _ in range(3):
            gb.set_variant(v)
            t, _, _ = gb.run(M, N, K, _lib.EPI_BIAS)
            best = max(best, t)
        cells.append("v%d %.0f" % (v, best))
    print(M, N, K, " | ".join(cells), flush=True)
gb.set_variant(0)
