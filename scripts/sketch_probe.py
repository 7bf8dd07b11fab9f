"""Where the 10M-row fit's sketch + binning time goes (bench.py's fit_breakdown 'sketch' / 'bin'):
has-missing scan, strided sample, compute_cuts, bin_matrix, each timed after a warm-up with device syncs."""
import time

import torch

from cobalt_smart_lender_ai_amd.dataio import synth
from cobalt_smart_lender_ai_amd.models import sketch
from cobalt_smart_lender_ai_amd.ops import gbdt_ops


def timed(fn, reps=5):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        out = fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3, out


def main():
    dev = torch.device("cuda", 0)
    X, _ = synth.make_lendingclub(10_000_000, seed=0, device=dev)
    ms_nan, hm = timed(lambda: torch.isnan(X).any(0))
    stride = sketch.sample_stride(X.shape[0], 1 << 18)
    ms_samp, samp = timed(lambda: sketch.local_sample(X, 0, stride).contiguous())
    ms_cuts, (cuts, nb) = timed(lambda: sketch.compute_cuts(samp, 256, None, hm))
    ms_bin, _ = timed(lambda: gbdt_ops.bin_matrix(X, cuts, nb))
    print(f"isnan.any {ms_nan:.3f} ms  sample {ms_samp:.3f} ms  compute_cuts {ms_cuts:.3f} ms  bin_matrix {ms_bin:.3f} ms")


if __name__ == "__main__":
    main()


def stages():
    """compute_cuts' stages on the 2^18-row sample (sort layouts, scans, searchsorted)."""
    dev = torch.device("cuda", 0)
    X, _ = synth.make_lendingclub(1 << 18, seed=0, device=dev)
    S, F = X.shape
    ms_sort0, srt = timed(lambda: torch.sort(X, dim=0))
    Xt = X.t().contiguous()
    ms_sort1, srt1 = timed(lambda: torch.sort(Xt, dim=1))
    ms_tr, _ = timed(lambda: X.t().contiguous())
    xs = srt1.values
    valid = ~torch.isnan(xs)
    ms_cum, cum = timed(lambda: torch.cumsum(valid.to(torch.int64), 1))
    k = torch.arange(1, 256, device=dev, dtype=torch.int64)
    W = cum[:, -1]
    ms_ss, _ = timed(lambda: torch.searchsorted((cum * 256).contiguous(), (k[None, :] * W[:, None]).contiguous(), right=True))
    print(f"sort dim0 {ms_sort0:.3f} ms  transpose {ms_tr:.3f}  sort dim1 {ms_sort1:.3f}  cumsum {ms_cum:.3f}  "
          f"searchsorted {ms_ss:.3f}")


if __name__ == "__main__":
    stages()
