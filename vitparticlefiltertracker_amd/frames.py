"""Frame sources — the metric's synthetic clip, plus plain readers for the "video
feed or images" the reference reads (README.md:42) but never ships. No cv2 / torchvision in this image, so the
readers are numpy: `.npy` clips, raw YUV4MPEG2 video (`.y4m`, what `ffmpeg -f yuv4mpegpipe` writes), binary PPM/PGM
images, and directories of frames. Compressed images (PNG, JPEG, BMP, TIFF, WebP) go through Pillow when it is
importable (it is in this image; imported on first use, with a clear error otherwise).

`prefetch(frames, depth)` decodes ahead on a host thread into pinned buffers, so a clip's decode (numpy YUV->RGB
of a 1080p frame is tens of ms) overlaps the previous frame's GPU work; `Tracker.track` takes the pinned tensor
and issues the H2D copy asynchronously on the current stream.

Clip: uint8 RGB frames; background uniform noise (numpy default_rng(seed)); a 64x64 textured target
(default_rng(seed + 1)) moving on a fixed trajectory, top-left x0 + t*v; bbox0 = (x0, y0, 64, 64).
"""
from __future__ import annotations

import glob
import os
import queue
import threading
from typing import Iterable, Iterator, Optional, Tuple

import numpy as np


def target_box(t: int, bbox0=(80, 80, 64, 64), velocity=(2, 1)) -> Tuple[int, int, int, int]:
    x0, y0, w, h = bbox0
    return x0 + velocity[0] * t, y0 + velocity[1] * t, w, h


def synthetic_clip(frames: int = 32, height: int = 224, width: int = 224, bbox0=(80, 80, 64, 64), seed: int = 7,
                   velocity=(2, 1)) -> np.ndarray:
    rng = np.random.default_rng(seed)
    bg = rng.integers(0, 256, size=(height, width, 3), dtype=np.uint8)
    tex = np.random.default_rng(seed + 1).integers(0, 256, size=(bbox0[3], bbox0[2], 3), dtype=np.uint8)
    out = np.empty((frames, height, width, 3), np.uint8)
    for t in range(frames):
        f = bg.copy()
        x, y, w, h = target_box(t, bbox0, velocity)
        xa, ya = max(0, x), max(0, y)
        xb, yb = min(width, x + w), min(height, y + h)
        if xa < xb and ya < yb:
            f[ya:yb, xa:xb] = tex[ya - y: yb - y, xa - x: xb - x]
        out[t] = f
    return out


# ---------------------------------------------------------------------------------------------- YUV4MPEG2
# Y'CbCr -> R'G'B' matrices (Kr, Kb); "limited" range = Y' in [16, 235], Cb/Cr in [16, 240] (what encoders emit
# unless told otherwise), "full" = all of [0, 255] (the C420jpeg convention of still-image pipelines).
_KRKB = {"bt601": (0.299, 0.114), "bt709": (0.2126, 0.0722)}


def yuv_to_rgb(y: np.ndarray, cb: np.ndarray, cr: np.ndarray, matrix: str = "bt601",
               full_range: bool = False) -> np.ndarray:
    """uint8 planes of equal shape [H][W] -> uint8 RGB [H][W][3] (round to nearest, clamped)."""
    kr, kb = _KRKB[matrix]
    kg = 1.0 - kr - kb
    yf = y.astype(np.float32)
    u = cb.astype(np.float32) - 128.0
    v = cr.astype(np.float32) - 128.0
    if not full_range:
        yf = (yf - 16.0) * (255.0 / 219.0)
        u *= 255.0 / 224.0
        v *= 255.0 / 224.0
    r = yf + (2.0 - 2.0 * kr) * v
    b = yf + (2.0 - 2.0 * kb) * u
    g = (yf - kr * r - kb * b) / kg
    out = np.empty(y.shape + (3,), np.uint8)
    for c, p in enumerate((r, g, b)):
        out[..., c] = np.clip(np.rint(p), 0, 255)
    return out


def rgb_to_yuv(rgb: np.ndarray, matrix: str = "bt601", full_range: bool = False):
    """uint8 RGB [H][W][3] -> (Y', Cb, Cr) uint8 planes [H][W] (the inverse of yuv_to_rgb; tests, writers)."""
    kr, kb = _KRKB[matrix]
    r, g, b = (rgb[..., c].astype(np.float32) for c in range(3))
    y = kr * r + (1.0 - kr - kb) * g + kb * b
    u = (b - y) / (2.0 - 2.0 * kb)
    v = (r - y) / (2.0 - 2.0 * kr)
    if not full_range:
        y = 16.0 + y * (219.0 / 255.0)
        u *= 224.0 / 255.0
        v *= 224.0 / 255.0
    q = lambda p: np.clip(np.rint(p), 0, 255).astype(np.uint8)   # noqa: E731
    return q(y), q(u + 128.0), q(v + 128.0)


def _y4m_header(fh) -> dict:
    line = fh.readline()
    if not line.startswith(b"YUV4MPEG2"):
        raise ValueError("not a YUV4MPEG2 stream")
    hdr = {"C": "420jpeg", "X": []}
    for tok in line.split()[1:]:
        tok = tok.decode("ascii")
        if tok[0] == "X":
            hdr["X"].append(tok[1:].upper())
        else:
            hdr[tok[0]] = tok[1:]
    if "W" not in hdr or "H" not in hdr:
        raise ValueError("YUV4MPEG2 header lacks W/H")
    if hdr.get("I", "p") not in ("p", "?"):
        raise ValueError(f"interlaced YUV4MPEG2 (I{hdr['I']}) is not supported")
    return hdr


def read_y4m(path, matrix: Optional[str] = None, full_range: Optional[bool] = None) -> Iterator[np.ndarray]:
    """Yield uint8 RGB frames of a progressive 8-bit YUV4MPEG2 file. Chroma: C420* (2x2 subsampled, upsampled by
    replication), C422 (2x1), C444, Cmono. Matrix defaults to BT.709 for frames wider than 1024 px (HD) and
    BT.601 otherwise; range defaults to limited, or full when the stream says XCOLORRANGE=FULL."""
    with open(path, "rb") as fh:
        hdr = _y4m_header(fh)
        W, H = int(hdr["W"]), int(hdr["H"])
        cs = hdr["C"]
        if matrix is None:
            matrix = "bt709" if W > 1024 else "bt601"
        if full_range is None:
            full_range = "COLORRANGE=FULL" in hdr["X"]
        if cs in ("420", "420jpeg", "420paldv", "420mpeg2"):
            cw, ch = (W + 1) // 2, (H + 1) // 2
        elif cs == "422":
            cw, ch = (W + 1) // 2, H
        elif cs == "444":
            cw, ch = W, H
        elif cs == "mono":
            cw = ch = 0
        else:
            raise ValueError(f"unsupported YUV4MPEG2 colourspace C{cs} (8-bit 420/422/444/mono only)")
        nbytes = W * H + 2 * cw * ch
        while True:
            tag = fh.readline()
            if not tag:
                return
            if not tag.startswith(b"FRAME"):
                raise ValueError("corrupt YUV4MPEG2 stream: FRAME marker expected")
            buf = fh.read(nbytes)
            if len(buf) != nbytes:
                raise ValueError("truncated YUV4MPEG2 frame")
            a = np.frombuffer(buf, np.uint8)
            y = a[: W * H].reshape(H, W)
            if cw == 0:
                yield np.repeat(y[..., None], 3, axis=2)
                continue
            cb = a[W * H: W * H + cw * ch].reshape(ch, cw)
            cr = a[W * H + cw * ch:].reshape(ch, cw)
            if (ch, cw) != (H, W):
                cb = np.repeat(np.repeat(cb, -(-H // ch), axis=0), -(-W // cw), axis=1)[:H, :W]
                cr = np.repeat(np.repeat(cr, -(-H // ch), axis=0), -(-W // cw), axis=1)[:H, :W]
            yield yuv_to_rgb(y, cb, cr, matrix, full_range)


class Y4MWriter:
    """Streaming YUV4MPEG2 writer (C444, or C420jpeg by 2x2 averaging): the output sink of main.py --video-out."""

    def __init__(self, path, fps: int = 30, chroma: str = "444", matrix: str = "bt601", full_range: bool = False):
        self.path, self.fps, self.matrix, self.full_range = path, fps, matrix, full_range
        self.tag = "444" if chroma == "444" else "420jpeg"
        self.fh = None
        self.shape = None

    def write(self, rgb: np.ndarray) -> None:
        H, W = rgb.shape[:2]
        if self.fh is None:
            self.shape = (H, W)
            extra = " XCOLORRANGE=FULL" if self.full_range else ""
            self.fh = open(self.path, "wb")
            self.fh.write(f"YUV4MPEG2 W{W} H{H} F{self.fps}:1 Ip A1:1 C{self.tag}{extra}\n".encode("ascii"))
        elif (H, W) != self.shape:
            raise ValueError("Y4MWriter: every frame must have the first frame's size")
        y, u, v = rgb_to_yuv(rgb, self.matrix, self.full_range)
        if self.tag != "444":
            def sub(p):
                pe = np.pad(p.astype(np.float32), ((0, H % 2), (0, W % 2)), mode="edge")
                s = pe.reshape(pe.shape[0] // 2, 2, pe.shape[1] // 2, 2).mean((1, 3))
                return np.clip(np.rint(s), 0, 255).astype(np.uint8)
            u, v = sub(u), sub(v)
        self.fh.write(b"FRAME\n")
        self.fh.write(y.tobytes() + u.tobytes() + v.tobytes())

    def close(self) -> None:
        if self.fh is not None:
            self.fh.close()
            self.fh = None

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()


def write_y4m(path, frames: Iterable[np.ndarray], fps: int = 30, chroma: str = "444", matrix: str = "bt601",
              full_range: bool = False) -> None:
    """Write RGB frames as YUV4MPEG2 (C444, or C420jpeg by 2x2 averaging) — fixtures and round-trip tests."""
    with Y4MWriter(path, fps, chroma, matrix, full_range) as w:
        for f in frames:
            w.write(f)


def draw_box(rgb: np.ndarray, box, color=(255, 0, 0), thickness: int = 2) -> np.ndarray:
    """A copy of the uint8 RGB frame with the (x, y, w, h) box outline drawn (clipped to the frame): the tracked
    position overlay of main.py --video-out."""
    out = np.array(rgb, dtype=np.uint8, copy=True)
    H, W = out.shape[:2]
    x0, y0 = int(round(box[0])), int(round(box[1]))
    x1, y1 = int(round(box[0] + box[2])) - 1, int(round(box[1] + box[3])) - 1
    t = max(1, int(thickness))
    col = np.asarray(color, dtype=np.uint8)
    for (ya, yb, xa, xb) in ((y0, y0 + t, x0, x1 + 1), (y1 - t + 1, y1 + 1, x0, x1 + 1),
                             (y0, y1 + 1, x0, x0 + t), (y0, y1 + 1, x1 - t + 1, x1 + 1)):
        ya, yb, xa, xb = max(ya, 0), min(yb, H), max(xa, 0), min(xb, W)
        if ya < yb and xa < xb:
            out[ya:yb, xa:xb] = col
    return out


# ---------------------------------------------------------------------------------------------- PPM / PGM
def _pnm_tokens(fh, n):
    out = []
    while len(out) < n:
        line = fh.readline()
        if not line:
            raise ValueError("truncated PNM header")
        out += line.split(b"#", 1)[0].split()
    return out


def read_pnm(path) -> np.ndarray:
    """Binary PPM (P6) -> uint8 RGB [H][W][3]; binary PGM (P5) -> grey replicated to RGB. maxval <= 255 only."""
    with open(path, "rb") as fh:
        magic, w, h, maxval = _pnm_tokens(fh, 4)
        w, h, maxval = int(w), int(h), int(maxval)
        if magic not in (b"P5", b"P6") or not 0 < maxval <= 255:
            raise ValueError(f"{path}: only 8-bit binary P5/P6 images are supported")
        c = 3 if magic == b"P6" else 1
        a = np.frombuffer(fh.read(w * h * c), np.uint8)
        if a.size != w * h * c:
            raise ValueError(f"{path}: truncated PNM raster")
    a = a.reshape(h, w, c)
    if maxval != 255:
        a = (a.astype(np.uint32) * 255 + maxval // 2) // maxval
    return np.ascontiguousarray(np.broadcast_to(a, (h, w, 3)), dtype=np.uint8)


def write_ppm(path, rgb: np.ndarray) -> None:
    h, w = rgb.shape[:2]
    with open(path, "wb") as fh:
        fh.write(f"P6\n{w} {h}\n255\n".encode("ascii"))
        fh.write(np.ascontiguousarray(rgb, dtype=np.uint8).tobytes())


# ---------------------------------------------------------------------------------------------- Pillow formats
_PIL_EXT = (".png", ".jpg", ".jpeg", ".bmp", ".tif", ".tiff", ".webp")


def _pil():
    try:
        from PIL import Image
    except ImportError as e:   # pragma: no cover - Pillow is in this image
        raise RuntimeError("reading or writing PNG / JPEG / BMP / TIFF / WebP frames needs Pillow (PIL), which is not "
                           "importable here; convert the frames to .ppm / .npy / .y4m") from e
    return Image


def read_image_pil(path) -> np.ndarray:
    """uint8[H][W][3] RGB of one PNG / JPEG / BMP / TIFF / WebP image (grey, palette and alpha images converted to
    RGB; the first frame of a multi-frame file)."""
    with _pil().open(path) as im:
        return np.ascontiguousarray(np.asarray(im.convert("RGB"), dtype=np.uint8))


def read_sequence_pil(path) -> Iterator[np.ndarray]:
    """Every frame of a multi-frame Pillow file (animated GIF / WebP / PNG, multi-page TIFF) as uint8[H][W][3] RGB;
    a single-frame image yields one frame."""
    with _pil().open(path) as im:
        for k in range(int(getattr(im, "n_frames", 1))):
            im.seek(k)
            yield np.ascontiguousarray(np.asarray(im.convert("RGB"), dtype=np.uint8))


def write_image_pil(path, rgb: np.ndarray, quality: int = 95) -> None:
    """Write uint8[H][W][3] RGB in the format the file suffix names (PNG lossless; JPEG at `quality`)."""
    im = _pil().fromarray(np.ascontiguousarray(rgb, dtype=np.uint8), "RGB")
    if os.fspath(path).lower().endswith((".jpg", ".jpeg")):
        im.save(path, quality=int(quality))
    else:
        im.save(path)


# ---------------------------------------------------------------------------------------------- dispatch
_IMAGE_EXT = (".npy", ".ppm", ".pgm", ".pnm") + _PIL_EXT


def _read_image(p) -> np.ndarray:
    low = p.lower()
    if low.endswith(".npy"):
        return np.load(p, allow_pickle=False)
    if low.endswith(_PIL_EXT):
        return read_image_pil(p)
    return read_pnm(p)


def iter_frames(source) -> Iterator[np.ndarray]:
    """Yield uint8[H][W][3] frames from a clip array, a `.npy` clip, a `.y4m` video, a single image (PPM/PGM, or
    PNG / JPEG / BMP / TIFF / WebP through Pillow; an animated GIF / WebP / PNG or a multi-page TIFF yields all its
    frames), or a directory of single-image frames (sorted by name)."""
    if isinstance(source, np.ndarray):
        arr = source if source.ndim == 4 else source[None]
        for f in arr:
            yield np.ascontiguousarray(f, dtype=np.uint8)
        return
    path = os.fspath(source)
    if os.path.isdir(path):
        files = sorted(p for p in glob.glob(os.path.join(path, "*")) if p.lower().endswith(_IMAGE_EXT))
        for p in files:
            yield np.ascontiguousarray(_read_image(p), dtype=np.uint8)
        return
    low = path.lower()
    if low.endswith(".y4m"):
        yield from read_y4m(path)
        return
    if low.endswith((".ppm", ".pgm", ".pnm")):
        yield read_pnm(path)
        return
    if low.endswith(_PIL_EXT + (".gif",)):   # a single image, or every frame of an animated / multi-page file
        yield from read_sequence_pil(path)
        return
    arr = np.load(path, mmap_mode="r", allow_pickle=False)
    for f in (arr if arr.ndim == 4 else arr[None]):
        yield np.ascontiguousarray(f, dtype=np.uint8)


def prefetch(frames: Iterable[np.ndarray], depth: int = 2, pin: bool = True) -> Iterator:
    """Decode ahead on one host thread. Yields torch uint8 tensors [H][W][3] in pinned memory (pin=True; ready
    for an asynchronous H2D copy) or the numpy frames themselves (pin=False). A ring of depth + 2 pinned buffers
    per frame shape is reused: a yielded tensor stays valid until the next one is taken (Tracker.track has
    synchronised on the frame's results by then); reader exceptions are re-raised in the consumer."""
    import torch

    if depth < 1:
        raise ValueError("depth must be >= 1")
    q: "queue.Queue" = queue.Queue(maxsize=depth)
    stop = threading.Event()
    END = object()
    ring_n = depth + 2
    rings = {}

    def work():
        k = 0
        try:
            for f in frames:
                if stop.is_set():
                    return
                f = np.ascontiguousarray(f, dtype=np.uint8)
                if pin:
                    ring = rings.setdefault(f.shape, [None] * ring_n)
                    if ring[k % ring_n] is None:
                        ring[k % ring_n] = torch.empty(f.shape, dtype=torch.uint8).pin_memory()
                    t = ring[k % ring_n]
                    t.numpy()[...] = f
                    f = t
                k += 1
                while not stop.is_set():
                    try:
                        q.put(f, timeout=0.1)
                        break
                    except queue.Full:
                        continue
            q.put(END)
        except BaseException as e:   # surfaced in the consumer
            q.put(e)

    th = threading.Thread(target=work, name="vpf-frame-prefetch", daemon=True)
    th.start()
    try:
        while True:
            item = q.get()
            if item is END:
                return
            if isinstance(item, BaseException):
                raise item
            yield item
    finally:
        stop.set()
        th.join(timeout=5)
