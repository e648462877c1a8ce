"""configs[1]'s one-launch quantizer under its calibration switches (FLC_QUANT_CAL bits: 1 non-temporal stores,
2 no grid exchange, 4 the memory traffic alone): kernel time by the live HIP-event probe and the step's wall time,
variants interleaved in one process.  Switch 1 is checked bit for bit against the default.  The switches exist only
in a calibration build: tools/build_variant.sh calib -DFLC_CALIB, then FLC_LIB=diag/lib_calib.so."""
import ctypes, os, sys, time
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch
from fl_sim_amd import codec, _lib

dev = torch.device("cuda", 0)
X = torch.randn(10, 417_482, generator=torch.Generator(device=dev).manual_seed(0), device=dev) * 1e-3


def run(c):
    return codec.quant_encode_auto(X, 0, 127, seed=0, counter=c)


def probe(name, fn, reps=200):
    for i in range(20):
        fn(i)
    torch.cuda.synchronize()
    _lib.call("flc_probe_set", name.encode())
    _lib.call("flc_probe_read", None, None)
    t0 = time.perf_counter()
    for i in range(reps):
        fn(i)
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) * 1e6 / reps
    t, c = ctypes.c_double(), ctypes.c_int64()
    _lib.call("flc_probe_read", ctypes.byref(t), ctypes.byref(c))
    _lib.call("flc_probe_set", None)
    return t.value / max(c.value, 1) * 1e3, wall


os.environ["FLC_QUANT_CAL"] = "0"
pk, out = run(7)
refs = [t.clone() for t in (pk.codes, out, pk.norms)]
os.environ["FLC_QUANT_CAL"] = "1"
pk, out = run(7)
torch.cuda.synchronize()
same = all(torch.equal(a.view(torch.uint8), b.view(torch.uint8)) for a, b in zip(refs, (pk.codes, out, pk.norms)))
print("nt stores bit-identical:", same, flush=True)
for rnd in range(3):
    for cal in (0, 1, 2, 4, 6):
        os.environ["FLC_QUANT_CAL"] = str(cal)
        k_us, wall = probe("quant_fused_encode_decode", run)
        print(f"round {rnd} cal={cal}: kernel {k_us:.2f} us  step {wall:.2f} us", flush=True)
