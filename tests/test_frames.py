"""Frame ingest: YUV4MPEG2 / PPM / PGM / .npy readers and the pinned prefetch thread.
CPU only. The colour conversion is checked against the BT.601 / BT.709 definitions at their anchor points, and
every reader by a write -> read round trip."""
import numpy as np
import pytest
import torch

from vitparticlefiltertracker_amd import frames as fr


def _clip(n=3, h=18, w=26, seed=0):
    return np.random.default_rng(seed).integers(0, 256, size=(n, h, w, 3), dtype=np.uint8)


@pytest.mark.parametrize("matrix", ["bt601", "bt709"])
@pytest.mark.parametrize("full", [False, True])
def test_yuv_anchor_points(matrix, full):
    """Black, white, grey and the six primaries/secondaries map to the expected code values."""
    lo, hi = (0, 255) if full else (16, 235)
    y = np.array([[lo, hi]], np.uint8)
    c = np.full_like(y, 128)
    rgb = fr.yuv_to_rgb(y, c, c, matrix, full)
    assert rgb[0, 0].tolist() == [0, 0, 0] and rgb[0, 1].tolist() == [255, 255, 255]
    prim = np.array([[[255, 0, 0], [0, 255, 0], [0, 0, 255], [0, 255, 255], [255, 0, 255], [255, 255, 0]]],
                    np.uint8)
    back = fr.yuv_to_rgb(*fr.rgb_to_yuv(prim, matrix, full), matrix, full)
    assert np.abs(back.astype(int) - prim).max() <= 3   # 8-bit Y'CbCr quantisation


@pytest.mark.parametrize("full", [False, True])
def test_y4m_444_round_trip(tmp_path, full):
    clip = _clip()
    p = tmp_path / "c.y4m"
    fr.write_y4m(p, clip, chroma="444", full_range=full)
    out = list(fr.iter_frames(str(p)))
    assert len(out) == len(clip)
    for a, b in zip(out, clip):
        assert a.shape == b.shape and a.dtype == np.uint8
        assert np.abs(a.astype(int) - b).max() <= (2 if full else 3)


def test_y4m_420_flat_blocks(tmp_path):
    """4:2:0 with odd sizes: constant-colour 2x2 blocks survive subsampling and replication upsampling."""
    h, w = 9, 13
    blocks = np.random.default_rng(3).integers(0, 256, size=((h + 1) // 2, (w + 1) // 2, 3), dtype=np.uint8)
    f = np.repeat(np.repeat(blocks, 2, 0), 2, 1)[:h, :w]
    p = tmp_path / "c420.y4m"
    fr.write_y4m(p, [f, f[::-1, ::-1].copy()], chroma="420")
    out = list(fr.read_y4m(p))
    assert len(out) == 2 and out[0].shape == (h, w, 3)
    assert np.abs(out[0].astype(int) - f).max() <= 3


def test_y4m_header_errors(tmp_path):
    p = tmp_path / "bad.y4m"
    p.write_bytes(b"YUV4MPEG2 W4 H2 It C420jpeg\n")
    with pytest.raises(ValueError, match="interlaced"):
        list(fr.read_y4m(p))
    p.write_bytes(b"YUV4MPEG2 W4 H2 C420p10\nFRAME\n")
    with pytest.raises(ValueError, match="colourspace"):
        list(fr.read_y4m(p))
    p.write_bytes(b"YUV4MPEG2 W4 H2 C444\nFRAME\n" + bytes(10))
    with pytest.raises(ValueError, match="truncated"):
        list(fr.read_y4m(p))
    p.write_bytes(b"YUV4MPEG2 W2 H2 Cmono\nFRAME\n" + bytes([0, 64, 128, 255]))
    (m,) = list(fr.read_y4m(p, full_range=True))
    assert m[..., 0].ravel().tolist() == [0, 64, 128, 255] and (m[..., 0] == m[..., 2]).all()


def test_pnm_and_directory(tmp_path):
    clip = _clip(4)
    d = tmp_path / "frames"
    d.mkdir()
    fr.write_ppm(d / "f000.ppm", clip[0])
    np.save(d / "f001.npy", clip[1])
    fr.write_ppm(d / "f002.ppm", clip[2])
    grey = clip[3, ..., 1]
    (d / "f003.pgm").write_bytes(b"P5\n# comment\n%d %d\n255\n" % (grey.shape[1], grey.shape[0]) + grey.tobytes())
    (d / "notes.txt").write_text("ignored")
    out = list(fr.iter_frames(str(d)))
    assert len(out) == 4
    for k in range(3):
        np.testing.assert_array_equal(out[k], clip[k])
    np.testing.assert_array_equal(out[3], np.repeat(grey[..., None], 3, 2))
    np.testing.assert_array_equal(fr.read_pnm(d / "f000.ppm"), clip[0])


def test_npy_clip_mmap(tmp_path):
    clip = _clip(5)
    np.save(tmp_path / "clip.npy", clip)
    out = list(fr.iter_frames(str(tmp_path / "clip.npy")))
    np.testing.assert_array_equal(np.stack(out), clip)


@pytest.mark.parametrize("pin", [False, True])
def test_prefetch_order_and_errors(pin):
    if pin and not torch.cuda.is_available():
        # pinned allocation needs the HIP runtime; exercise the same ring/thread logic unpinned on CPU
        pin = False
    clip = _clip(7)
    got = []
    for f in fr.prefetch(iter(clip), depth=2, pin=pin):
        got.append(np.array(f.numpy() if isinstance(f, torch.Tensor) else f))   # copy: the ring slot is reused
    np.testing.assert_array_equal(np.stack(got), clip)

    def broken():
        yield clip[0]
        raise OSError("disk gone")
    it = fr.prefetch(broken(), depth=1, pin=False)
    next(it)
    with pytest.raises(OSError, match="disk gone"):
        next(it)


def test_prefetch_early_close():
    """Abandoning the consumer stops the reader thread (no hang at interpreter exit)."""
    it = fr.prefetch(iter(_clip(50)), depth=1, pin=False)
    next(it)
    it.close()


def test_draw_box_outline_and_clipping():
    img = np.zeros((20, 30, 3), np.uint8)
    out = fr.draw_box(img, (5, 4, 10, 8), color=(9, 8, 7), thickness=2)
    assert img.sum() == 0                                     # input untouched
    on = (out == np.array([9, 8, 7], np.uint8)).all(axis=2)
    assert on[4, 5] and on[4, 14] and on[11, 5] and on[11, 14] and on[5, 6]   # corners and the 2-px border
    assert not on[7, 8] and not on[3, 5] and not on[12, 5]   # interior and outside stay black
    clipped = fr.draw_box(img, (-5, -5, 12, 12), thickness=1)   # partly outside: clipped, no error
    assert clipped[6, 0:7].any() and clipped.shape == img.shape


def test_y4m_writer_streams(tmp_path):
    clip = _clip(4, 10, 12)
    p = tmp_path / "w.y4m"
    with fr.Y4MWriter(p) as w:
        for f in clip:
            w.write(f)
    back = list(fr.read_y4m(p))
    assert len(back) == 4 and np.abs(back[2].astype(int) - clip[2]).max() <= 3
    with pytest.raises(ValueError, match="size"):
        with fr.Y4MWriter(tmp_path / "x.y4m") as w:
            w.write(clip[0])
            w.write(clip[0][:5])


def test_pillow_images_and_directory(tmp_path):
    """PNG (lossless: exact), JPEG (lossy: close), BMP and a grey PNG through Pillow, alone and mixed with PPM / .npy
    frames in one directory (sorted by name); and the writer main.py's --frame-format uses."""
    clip = _clip(5)
    d = tmp_path / "mixed"
    d.mkdir()
    fr.write_image_pil(d / "f000.png", clip[0])
    fr.write_ppm(d / "f001.ppm", clip[1])
    yy, xx = np.mgrid[: clip.shape[1], : clip.shape[2]]
    smooth = np.stack([xx * 9, yy * 13, (xx + yy) * 5], 2).astype(np.uint8)   # JPEG is meant for smooth images
    fr.write_image_pil(d / "f002.jpg", smooth, quality=98)
    fr.write_image_pil(d / "f003.bmp", clip[3])
    grey = clip[4, ..., 0]
    from PIL import Image
    Image.fromarray(grey, "L").save(d / "f004.png")
    out = list(fr.iter_frames(str(d)))
    assert len(out) == 5 and all(o.dtype == np.uint8 and o.shape == clip[0].shape for o in out)
    np.testing.assert_array_equal(out[0], clip[0])
    np.testing.assert_array_equal(out[1], clip[1])
    assert np.abs(out[2].astype(int) - smooth.astype(int)).mean() < 3     # lossy
    np.testing.assert_array_equal(out[3], clip[3])
    np.testing.assert_array_equal(out[4], np.repeat(grey[..., None], 3, 2))
    np.testing.assert_array_equal(next(fr.iter_frames(str(d / "f000.png"))), clip[0])


def test_animated_gif_and_multipage_tiff(tmp_path):
    """An animated GIF (palette: lossy on noise, exact on a few flat colours) and a multi-page TIFF (lossless) read as
    clips, every frame in order."""
    from PIL import Image
    clip = _clip(4)
    pages = [Image.fromarray(f, "RGB") for f in clip]
    pages[0].save(tmp_path / "clip.tif", save_all=True, append_images=pages[1:])
    out = list(fr.iter_frames(str(tmp_path / "clip.tif")))
    assert len(out) == 4
    for k in range(4):
        np.testing.assert_array_equal(out[k], clip[k])
    flat = np.zeros((4, 20, 30, 3), np.uint8)
    for k in range(4):
        flat[k, :, : 10 + 5 * k] = (255, 0, 0)          # a growing red bar on black
    gif = [Image.fromarray(f, "RGB") for f in flat]
    gif[0].save(tmp_path / "clip.gif", save_all=True, append_images=gif[1:], duration=40, loop=0)
    out = list(fr.iter_frames(str(tmp_path / "clip.gif")))
    assert len(out) == 4
    for k in range(4):
        np.testing.assert_array_equal(out[k], flat[k])
