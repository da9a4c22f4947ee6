"""Per-launch cost of back-to-back dependent kernels on one stream, queued behind a spin kernel
(host enqueue hidden): torch elementwise kernels vs this library's kernels through the C ABI."""
import sys
from pathlib import Path

REPO = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(REPO / "contrast-gan-3d_amd"))
import torch  # noqa: E402


def per_launch(fn, n=400):
    for _ in range(5):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda._sleep(40_000_000)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return round(e0.elapsed_time(e1) * 1e3 / n, 2)


def main():
    from cgan3d_amd import _lib
    lib = _lib.load()
    s = torch.cuda.current_stream().cuda_stream
    x = torch.zeros(1, device="cuda")
    big = torch.zeros(1 << 20, device="cuda")
    hyper = torch.zeros(8, device="cuda")
    y = torch.zeros(256, device="cuda")
    print("torch tiny add", per_launch(lambda: x.add_(1)))
    print("torch 4MB add", per_launch(lambda: big.add_(1)))
    print("cgan3d_adam_tick (1 thread)", per_launch(lambda: lib.cgan3d_adam_tick(hyper.data_ptr(), s)))
    print("cgan3d_tanh_backward (256)", per_launch(
        lambda: lib.cgan3d_tanh_backward(y.data_ptr(), y.data_ptr(), y.data_ptr(), 256, s)))
    print("alternating torch add / adam_tick", per_launch(
        lambda: (x.add_(1), lib.cgan3d_adam_tick(hyper.data_ptr(), s))))


if __name__ == "__main__":
    main()
