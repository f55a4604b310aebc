"""GPU: the reference-compatible codec CLI (dct3d_codec encode/decode, the boundary's callers) end to
end.  The .bin must be byte-identical to the reference C encoder's entropy stage applied to the
Java-semantics coefficients, and the decoded raw file must equal the Java-semantics decode."""
import os
import subprocess

import numpy as np
import pytest

from test_host_codec import reference_entropy_encode

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("host_eg,batch", [("0", "2"), ("1", "2"), ("0", "1"), ("0", "16")])
@pytest.mark.parametrize("w,h,frames,kind", [(64, 64, 16, "ramp"), (320, 240, 24, "uniform"), (64, 48, 12, "ramp"),
                                             (136, 72, 24, "ramp")])  # 153 cubes a stack
def test_cli_encode_decode(pkg, plan8, tmp_path, w, h, frames, kind, host_eg, batch):
    """host_eg "0": DCT + quantisation + Exp-Golomb on the device, one deflate call per batch;
    "1": the reference's split (ints over PCIe, Exp-Golomb on the host, one deflate call per stack).
    Both must give the reference encoder's bytes."""
    fr = pkg.synthetic.frames(w, h, frames, kind=kind)
    n_stacks = (frames + 7) // 8
    padded = np.zeros((n_stacks * 8, h, w), np.uint8)
    padded[:frames] = fr                              # short last stack is zero-filled
    raw = tmp_path / "in.raw"
    raw.write_bytes(fr.tobytes())
    binf, outf = tmp_path / "out.bin", tmp_path / "out.raw"
    env = dict(os.environ, DCT3D_CODEC_BATCH=batch, DCT3D_CODEC_HOST_EG=host_eg)
    r = subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), "1"],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    q = plan8.encode_q(padded).reshape(-1)
    assert binf.read_bytes() == reference_entropy_encode(q, w, h, n_stacks, 8)
    r = subprocess.run([pkg.CLI_PATH, "decode", str(binf), str(outf), str(w), str(h), str(frames), "1"],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    dec = np.frombuffer(outf.read_bytes(), np.uint8).reshape(n_stacks * 8, h, w)
    assert np.array_equal(dec, plan8.decode_q(q.reshape(-1, 8, 8, 8), w, h, n_stacks * 8))


@pytest.mark.parametrize("devices,batch", [("1,1", "1"), ("1,1,1", "2"), ("1,1", "16")])
@pytest.mark.parametrize("w,h,frames,kind", [(64, 64, 40, "ramp"), (320, 240, 24, "uniform")])
def test_cli_multi_device(pkg, plan8, tmp_path, w, h, frames, kind, devices, batch):
    """encode_multi / decode_multi (a device list; one box has one GPU, so the list repeats it: one
    context and host thread per entry).  The batches' streams, coded from a zero carry on their own
    contexts and joined in order, must give the reference encoder's bytes; the chained multi-context
    decode must give the Java-semantics decode."""
    fr = pkg.synthetic.frames(w, h, frames, kind=kind)
    n_stacks = (frames + 7) // 8
    padded = np.zeros((n_stacks * 8, h, w), np.uint8)
    padded[:frames] = fr
    raw = tmp_path / "in.raw"
    raw.write_bytes(fr.tobytes())
    binf, outf = tmp_path / "out.bin", tmp_path / "out.raw"
    env = dict(os.environ, DCT3D_CODEC_BATCH=batch)
    r = subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), devices],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    assert r.stdout.count("Frames processed") == n_stacks
    q = plan8.encode_q(padded).reshape(-1)
    assert binf.read_bytes() == reference_entropy_encode(q, w, h, n_stacks, 8)
    r = subprocess.run([pkg.CLI_PATH, "decode", str(binf), str(outf), str(w), str(h), str(frames), devices],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    dec = np.frombuffer(outf.read_bytes(), np.uint8).reshape(n_stacks * 8, h, w)
    assert np.array_equal(dec, plan8.decode_q(q.reshape(-1, 8, 8, 8), w, h, n_stacks * 8))


def test_cli_multi_device_depth4(pkg, plan4, tmp_path):
    """encode_multi / decode_multi at block depth 4: the batches' streams joined behind the running partial
    byte give the single-device .bin, and the chained decode the Java-semantics decode."""
    w, h, frames = 64, 32, 20
    fr = pkg.synthetic.frames(w, h, frames, kind="uniform")
    n_stacks = (frames + 3) // 4
    raw, b1, bm, outf = tmp_path / "in.raw", tmp_path / "one.bin", tmp_path / "multi.bin", tmp_path / "o.raw"
    raw.write_bytes(fr.tobytes())
    env = dict(os.environ, DCT3D_CODEC_BATCH="2")
    for binf, dev in ((b1, "1"), (bm, "1,1,1")):
        r = subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), dev, "4"],
                           capture_output=True, text=True, env=env)
        assert r.returncode == 0, r.stdout + r.stderr
    assert bm.read_bytes() == b1.read_bytes()
    r = subprocess.run([pkg.CLI_PATH, "decode", str(bm), str(outf), str(w), str(h), str(frames), "1,1", "4"],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 0, r.stdout + r.stderr
    padded = np.zeros((n_stacks * 4, h, w), np.uint8)
    padded[:frames] = fr
    q = plan4.encode_q(padded)
    dec = np.frombuffer(outf.read_bytes(), np.uint8).reshape(n_stacks * 4, h, w)
    assert np.array_equal(dec, plan4.decode_q(q, w, h, n_stacks * 4))


def test_cli_multi_device_truncated_and_bad_device(pkg, tmp_path):
    w, h, frames = 64, 48, 24
    fr = pkg.synthetic.frames(w, h, frames, kind="uniform")
    raw, binf, outf = tmp_path / "in.raw", tmp_path / "o.bin", tmp_path / "o.raw"
    raw.write_bytes(fr.tobytes())
    env = dict(os.environ, DCT3D_CODEC_BATCH="1")
    assert subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), "1,1"],
                          capture_output=True, env=env).returncode == 0
    data = binf.read_bytes()
    binf.write_bytes(data[: len(data) // 2])
    r = subprocess.run([pkg.CLI_PATH, "decode", str(binf), str(outf), str(w), str(h), str(frames), "1,1"],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 1 and "Truncated or corrupt" in r.stdout
    r = subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), "1,99"],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 1 and "device 99" in r.stdout


def test_cli_depth4(pkg, plan4, tmp_path):
    w, h, frames = 64, 32, 8
    fr = pkg.synthetic.frames(w, h, frames, kind="uniform")
    raw, binf, outf = tmp_path / "in.raw", tmp_path / "o.bin", tmp_path / "o.raw"
    raw.write_bytes(fr.tobytes())
    assert subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), "1", "4"],
                          capture_output=True).returncode == 0
    assert subprocess.run([pkg.CLI_PATH, "decode", str(binf), str(outf), str(w), str(h), str(frames), "1", "4"],
                          capture_output=True).returncode == 0
    q = plan4.encode_q(fr)
    dec = np.frombuffer(outf.read_bytes(), np.uint8).reshape(frames, h, w)
    assert np.array_equal(dec, plan4.decode_q(q, w, h, frames))


@pytest.mark.parametrize("host_eg", ["0", "1"])
def test_cli_decode_truncated_input_fails_cleanly(pkg, tmp_path, host_eg):
    w, h, frames = 64, 48, 16
    fr = pkg.synthetic.frames(w, h, frames, kind="uniform")
    raw, binf, outf = tmp_path / "in.raw", tmp_path / "o.bin", tmp_path / "o.raw"
    raw.write_bytes(fr.tobytes())
    env = dict(os.environ, DCT3D_CODEC_HOST_EG=host_eg)
    assert subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), "1"],
                          capture_output=True, env=env).returncode == 0
    data = binf.read_bytes()
    binf.write_bytes(data[: len(data) // 2])
    r = subprocess.run([pkg.CLI_PATH, "decode", str(binf), str(outf), str(w), str(h), str(frames), "1"],
                       capture_output=True, text=True, env=env)
    assert r.returncode == 1 and "Truncated or corrupt" in r.stdout


def test_cli_multi_device_distinct_gpus(pkg, plan8, tmp_path):
    """encode_multi / decode_multi over two DISTINCT devices: one context, host thread and
    per-device raster allocation on each GPU.  The round's boxes have one GPU, so this runs only where the
    CLI lists two or more devices (the driver's 8-GPU node); elsewhere it skips."""
    r = subprocess.run([pkg.CLI_PATH, "list_devices"], capture_output=True, text=True, timeout=120)
    n_dev = sum(1 for line in r.stdout.splitlines() if " - HIP device " in line)
    if n_dev < 2:
        pytest.skip(f"{n_dev} HIP device(s): distinct-device multi-GPU codec needs two")
    w, h, frames = 320, 240, 40
    fr = pkg.synthetic.frames(w, h, frames, kind="ramp")
    n_stacks = frames // 8
    raw, b1, b2, o2 = tmp_path / "in.raw", tmp_path / "one.bin", tmp_path / "two.bin", tmp_path / "two.raw"
    raw.write_bytes(fr.tobytes())
    env = dict(os.environ, DCT3D_CODEC_BATCH="1")
    for binf, dev in ((b1, "1"), (b2, "1,2")):
        r = subprocess.run([pkg.CLI_PATH, "encode", str(raw), str(binf), str(w), str(h), str(frames), dev],
                           capture_output=True, text=True, env=env, timeout=300)
        assert r.returncode == 0, r.stdout + r.stderr
    assert b2.read_bytes() == b1.read_bytes()
    r = subprocess.run([pkg.CLI_PATH, "decode", str(b2), str(o2), str(w), str(h), str(frames), "2,1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stdout + r.stderr
    q = plan8.encode_q(fr)
    dec = np.frombuffer(o2.read_bytes(), np.uint8).reshape(frames, h, w)
    assert np.array_equal(dec, plan8.decode_q(q.reshape(-1, 8, 8, 8), w, h, frames))
