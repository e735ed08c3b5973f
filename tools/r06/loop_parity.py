"""Parity of a conv_pipe experiment policy (measurement library, YOLOMI_LIB=libyolomi_exp.so): runs
tests/test_gpu_conv.py's forced-pipe checks (fp16 forward + BN partials, bf16 data gradient overwrite / accumulate,
views) on every PIPE shape with SETTER=VALUE applied.   usage: python tools/r06/loop_parity.py ym_conv_set_pipe_loop 1"""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[2]
for p in (str(ROOT), str(ROOT / "yolo-scratch_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)


def main():
    import test_gpu_conv as T
    from yolomi._lib import lib
    setter, val = sys.argv[1], int(sys.argv[2])
    getattr(lib(), setter)(val)
    for shape in T.PIPE:
        T._views_fwd_dgrad_check(shape, lib().ym_conv_set_pipe, 2, 2)
        print("ok", shape, flush=True)
    getattr(lib(), setter)(0)
    print("all shapes ok")


if __name__ == "__main__":
    main()
