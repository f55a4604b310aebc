"""End-to-end codec timing (run on the GPU box): the reference-compatible CLI on a synthetic 1080p raw
file, Exp-Golomb on the host (the reference's split: quantised ints over PCIe) vs on the device (only
the stream crosses PCIe), encode and decode; both must write the same .bin / frames.  Every CLI run also
reports its per-stage wall seconds (DCT3D_CODEC_TIMING=1, codec.c: ctx create, read, device, stream
fetch, deflate + write / read + inflate, device, write) under "stages".  One JSON line."""
import importlib, json, os, subprocess, sys, tempfile, time, zlib

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
pkg = importlib.import_module("3ddctvideoencoding_amd")

W, H = 1920, 1080
F = int(os.environ.get("E2E_FRAMES", "64"))
tmp = tempfile.mkdtemp(dir=os.environ.get("TMPDIR", "/tmp"))
raw = os.path.join(tmp, "in.raw")
with open(raw, "wb") as f:
    for s in range(0, F, 8):
        f.write(pkg.synthetic.frames(W, H, min(8, F - s), kind="ramp", frame0=s).tobytes())
res = {"frames": F, "width": W, "height": H, "raw_MB": W * H * F / 1e6, "stages": {}}


def run_cli(name, args, env):
    env = dict(env, DCT3D_CODEC_TIMING="1")
    t0 = time.perf_counter()
    r = subprocess.run([pkg.CLI_PATH] + args, capture_output=True, text=True, env=env)
    dt = time.perf_counter() - t0
    assert r.returncode == 0, r.stdout + r.stderr
    st = [json.loads(l) for l in r.stderr.splitlines() if l.startswith('{"stage_s"')]
    res["stages"][name] = dict(st[-1], process_s=dt) if st else {"process_s": dt}
    return dt

bins = {}
for mode in ("1", "0"):
    env = dict(os.environ, DCT3D_CODEC_HOST_EG=mode)
    out = os.path.join(tmp, f"out{mode}.bin")
    dt = run_cli("encode_host_eg" if mode == "1" else "encode", ["encode", raw, out, str(W), str(H), str(F), "1"], env)
    bins[mode] = open(out, "rb").read()
    res["encode_host_eg_s" if mode == "1" else "encode_device_eg_s"] = dt
res["bin_identical"] = bins["0"] == bins["1"]
# optional parallel deflate: a different .bin, the same inflated payload
T = int(os.environ.get("E2E_DEFLATE_THREADS", "16"))
env = dict(os.environ, DCT3D_CODEC_HOST_EG="0", DCT3D_CODEC_DEFLATE_THREADS=str(T))
outp = os.path.join(tmp, "outp.bin")
res["encode_parallel_deflate_s"] = run_cli("encode_parallel_deflate", ["encode", raw, outp, str(W), str(H), str(F), "1"], env)
binp = open(outp, "rb").read()
res["deflate_threads"] = T
res["parallel_bin_MB"] = len(binp) / 1e6
res["parallel_payload_identical"] = zlib.decompress(binp) == zlib.decompress(bins["0"])
res["encode_parallel_deflate_fps"] = F / res["encode_parallel_deflate_s"]
res["bin_MB"] = len(bins["0"]) / 1e6
decs = {}
for mode in ("1", "0", "p"):
    env = dict(os.environ, DCT3D_CODEC_HOST_EG="1" if mode == "1" else "0")
    src = os.path.join(tmp, "outp.bin" if mode == "p" else "out0.bin")
    dec = os.path.join(tmp, f"dec{mode}.raw")
    key = {"1": "decode_host_eg", "0": "decode", "p": "decode_parallel_bin"}[mode]
    res[key + "_s"] = run_cli(key, ["decode", src, dec, str(W), str(H), str(F), "1"], env)
    decs[mode] = open(dec, "rb").read()
res["decoded_identical"] = decs["0"] == decs["1"] == decs["p"]
res["encode_device_eg_fps"] = F / res["encode_device_eg_s"]
res["encode_host_eg_fps"] = F / res["encode_host_eg_s"]
res["decode_fps"] = F / res["decode_s"]
res["decode_host_eg_fps"] = F / res["decode_host_eg_s"]
print(json.dumps(res))
