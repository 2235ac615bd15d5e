"""WavLM conv layer 0 + GroupNorm + GELU at the bench's shape (B = 32 utterances of 10 s at 16 kHz, 512 channels,
kernel 10, stride 5, bf16 output): HIP-event time per call (statistics + affine + apply launches) and the rate of
the 1.05 GB bf16 output. FDDM_CONV0_VALU=1 selects the VALU recompute kernel."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "fddm-asr_amd"))
import torch  # noqa: E402

from fddm_hip import ops  # noqa: E402


def main():
    dev = torch.device("cuda:0")
    B, nsamp, C, K, S = 32, 160000, 512, 10, 5
    wave = torch.randn(B, nsamp, device=dev) * 0.1
    w = torch.randn(C, K, device=dev) * 0.3
    gamma, beta = torch.ones(C, device=dev), torch.zeros(C, device=dev)
    f = lambda: ops.conv0_gn_gelu(wave, w, gamma, beta, torch.bfloat16, C, K, S)  # noqa: E731
    for _ in range(5):
        f()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 30
    s.record()
    for _ in range(n):
        f()
    e.record()
    torch.cuda.synchronize()
    t = s.elapsed_time(e) / n * 1e3
    T0 = (nsamp - K) // S + 1
    byt = B * T0 * C * 2
    print(f"conv0 [{'valu' if os.environ.get('FDDM_CONV0_VALU') else 'mfma'}] {t:7.1f} us  {byt / t / 1e3:6.0f} GB/s",
          flush=True)


if __name__ == "__main__":
    main()
