"""Data formats either side of the sampler.

* HEALPix FITS maps: ``read_map`` / ``write_map`` -- the subset of
  healpy.read_map / write_map the reference uses (``hp.read_map(mask_path)``
  and ``hp.read_map(mask_path, 0)``, config.py:126, ClsSampler.py:31,
  NonCenteredGibbs.py:288, main_polarization.py:53).  A minimal FITS reader
  (FITS 4.0 standard: 2880-byte blocks, 80-byte cards, big-endian binary
  tables) for full-sky IMPLICIT maps in RING or NESTED order; NESTED maps
  are returned in RING order as healpy does by default.
* ``ud_grade`` -- healpy.ud_grade (degrade = mean of the non-UNSEEN
  sub-pixels, ``pess`` = UNSEEN if any is; upgrade = replicate), the
  mask-resolution step of config.py:126 / ClsSampler.py:31.
* ``nest2ring`` / ``ring2nest`` -- the HEALPix pixel-index conversions
  (Gorski et al. 2005, ApJ 622, 759; the published xyf <-> ring mapping).
* the run record of main_polarization.py:172-185 (``run_record``) and the
  dataset dict of main_polarization.py:77-81 (``dataset_record``), written
  as plain-array ``.npz`` archives (``save_npz`` / ``load_npz``, no
  pickling: None values are stored as empty arrays and flagged).

healpy / astropy are absent here; this module is host-side I/O (setup
time), not a compute path.  Parity: the FITS layer is pinned by the FITS
standard and round trips (no reference FITS file ships with the reference);
nest2ring by pixel-centre geometry against the RING pixelisation.
"""
import math
import os

import numpy as np

UNSEEN = -1.6375e30          # healpy.UNSEEN
_BLOCK = 2880

# ---------------------------------------------------------------------------------------
# HEALPix NESTED <-> RING
# ---------------------------------------------------------------------------------------
_JRLL = np.array([2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4], dtype=np.int64)
_JPLL = np.array([1, 3, 5, 7, 0, 2, 4, 6, 1, 3, 5, 7], dtype=np.int64)


def _compress_bits(v):
    """keep the even bits of v (de-interleave), vectorised."""
    v = v & 0x5555555555555555
    v = (v | (v >> 1)) & 0x3333333333333333
    v = (v | (v >> 2)) & 0x0F0F0F0F0F0F0F0F
    v = (v | (v >> 4)) & 0x00FF00FF00FF00FF
    v = (v | (v >> 8)) & 0x0000FFFF0000FFFF
    v = (v | (v >> 16)) & 0x00000000FFFFFFFF
    return v


def _check_nside(nside):
    nside = int(nside)
    if nside < 1 or (nside & (nside - 1)) != 0:
        raise ValueError("nside must be a power of 2 (NESTED ordering)")
    return nside


def nest2ring(nside, ipix):
    """NESTED pixel index -> RING pixel index (vectorised, int64)."""
    nside = _check_nside(nside)
    ipix = np.asarray(ipix, dtype=np.int64)
    npface = nside * nside
    npix = 12 * npface
    if np.any((ipix < 0) | (ipix >= npix)):
        raise ValueError("pixel index out of range")
    face = ipix // npface
    ipf = ipix % npface
    ix = _compress_bits(ipf)
    iy = _compress_bits(ipf >> 1)
    nl4 = 4 * nside
    ncap = 2 * nside * (nside - 1)
    jr = _JRLL[face] * nside - ix - iy - 1
    nr = np.where(jr < nside, jr, np.where(jr > 3 * nside, nl4 - jr, nside))
    n_before = np.where(jr < nside, 2 * nr * (nr - 1),
                        np.where(jr > 3 * nside, npix - 2 * (nr + 1) * nr, ncap + (jr - nside) * nl4))
    kshift = np.where((jr >= nside) & (jr <= 3 * nside), (jr - nside) & 1, 0)
    jp = (_JPLL[face] * nr + ix - iy + 1 + kshift) // 2
    jp = np.where(jp > nl4, jp - nl4, jp)
    jp = np.where(jp < 1, jp + nl4, jp)
    return n_before + jp - 1


_R2N_CACHE = {}


def ring2nest(nside, ipix):
    """RING pixel index -> NESTED pixel index (inverse permutation of nest2ring)."""
    nside = _check_nside(nside)
    perm = _R2N_CACHE.get(nside)
    if perm is None:
        npix = 12 * nside * nside
        perm = np.empty(npix, dtype=np.int64)
        perm[nest2ring(nside, np.arange(npix, dtype=np.int64))] = np.arange(npix, dtype=np.int64)
        if len(_R2N_CACHE) > 4:
            _R2N_CACHE.clear()
        _R2N_CACHE[nside] = perm
    return perm[np.asarray(ipix, dtype=np.int64)]


def npix2nside(npix):
    nside = int(round(math.sqrt(npix / 12.0)))
    if 12 * nside * nside != npix:
        raise ValueError("not a HEALPix map size: %d" % npix)
    return nside


def reorder(m, r2n=False, n2r=False):
    """healpy.reorder (last axis)."""
    m = np.asarray(m)
    if r2n == n2r:
        raise ValueError("give exactly one of r2n / n2r")
    npix = m.shape[-1]
    idx = nest2ring(npix2nside(npix), np.arange(npix, dtype=np.int64))
    if r2n:                       # nested[p] = ring[nest2ring(p)]
        return m[..., idx]
    out = np.empty_like(m)
    out[..., idx] = m
    return out


# ---------------------------------------------------------------------------------------
# ud_grade
# ---------------------------------------------------------------------------------------
def ud_grade(map_in, nside_out, pess=False, order_in="RING", order_out=None, power=None, dtype=None):
    """healpy.ud_grade: change the resolution of a map.

    Degrading averages the (nside_in/nside_out)^2 NESTED children of every
    output pixel, skipping UNSEEN (``pess``: UNSEEN as soon as one child is);
    upgrading copies each pixel to its children.  ``power`` multiplies by
    (nside_out/nside_in)^power."""
    m = np.asarray(map_in, dtype=np.float64 if dtype is None else dtype)
    nside_in = _check_nside(npix2nside(m.shape[-1]))
    nside_out = _check_nside(nside_out)
    order_out = order_in if order_out is None else order_out
    if order_in.upper() not in ("RING", "NESTED") or order_out.upper() not in ("RING", "NESTED"):
        raise ValueError("order must be RING or NESTED")
    nest = m if order_in.upper() == "NESTED" else reorder(m, r2n=True)
    if nside_out < nside_in:
        r = (nside_in // nside_out) ** 2
        ch = nest.reshape(nest.shape[:-1] + (12 * nside_out * nside_out, r))
        seen = (ch != UNSEEN) & np.isfinite(ch)
        nseen = seen.sum(axis=-1)
        tot = np.where(seen, ch, 0.0).sum(axis=-1)
        out = np.where(nseen > 0, tot / np.maximum(nseen, 1), UNSEEN)
        if pess:
            out = np.where(nseen == r, out, UNSEEN)
    elif nside_out > nside_in:
        out = np.repeat(nest, (nside_out // nside_in) ** 2, axis=-1)
    else:
        out = nest.copy()
    if power is not None:
        ratio = (float(nside_out) / float(nside_in)) ** float(power)
        out = np.where(out != UNSEEN, out * ratio, UNSEEN)
    out = out.astype(m.dtype, copy=False)
    return out if order_out.upper() == "NESTED" else reorder(out, n2r=True)


# ---------------------------------------------------------------------------------------
# FITS
# ---------------------------------------------------------------------------------------
_TFORM = {"L": "u1", "B": "u1", "I": ">i2", "J": ">i4", "K": ">i8", "E": ">f4", "D": ">f8"}


def _parse_value(v):
    v = v.strip()
    if v.startswith("'"):
        i, out = 1, []
        while i < len(v):
            if v[i] == "'":
                if i + 1 < len(v) and v[i + 1] == "'":
                    out.append("'")
                    i += 2
                    continue
                break
            out.append(v[i])
            i += 1
        return "".join(out).rstrip()
    if "/" in v:
        v = v.split("/", 1)[0].strip()
    if v in ("T", "F"):
        return v == "T"
    try:
        return int(v)
    except ValueError:
        try:
            return float(v.replace("D", "E"))
        except ValueError:
            return v


def _read_header(f):
    cards, order = {}, []
    while True:
        blk = f.read(_BLOCK)
        if len(blk) < _BLOCK:
            raise ValueError("truncated FITS header")
        for i in range(0, _BLOCK, 80):
            card = blk[i:i + 80].decode("ascii", errors="replace")
            key = card[:8].strip()
            if key == "END":
                return cards, order
            if card[8:10] == "= " and key:
                cards[key] = _parse_value(card[10:])
                order.append(key)


def _skip_data(f, h):
    naxis = int(h.get("NAXIS", 0))
    n = 0
    if naxis > 0:
        n = abs(int(h.get("BITPIX", 8))) // 8
        for k in range(1, naxis + 1):
            n *= int(h["NAXIS%d" % k])
        n = (n + int(h.get("PCOUNT", 0))) * int(h.get("GCOUNT", 1))
    f.seek((n + _BLOCK - 1) // _BLOCK * _BLOCK, os.SEEK_CUR)


def _column_dtype(h):
    fields = []
    for k in range(1, int(h["TFIELDS"]) + 1):
        tf = str(h["TFORM%d" % k]).strip()
        j = 0
        while j < len(tf) and tf[j].isdigit():
            j += 1
        rep = int(tf[:j]) if j else 1
        if j >= len(tf) or tf[j] not in _TFORM:
            raise ValueError("unsupported FITS column type %r" % tf)
        fields.append(("c%d" % k, _TFORM[tf[j]], (rep,)))
    return np.dtype(fields)


def read_map(filename, field=0, dtype=np.float64, nest=False, hdu=1, h=False):
    """healpy.read_map for full-sky (IMPLICIT) HEALPix binary tables.

    ``field``: column index or tuple of indices; RING order unless
    ``nest=True``; ``h=True`` also returns the extension header cards."""
    with open(filename, "rb") as f:
        hdr, _ = _read_header(f)
        if not hdr.get("SIMPLE", False):
            raise ValueError("not a FITS file")
        _skip_data(f, hdr)
        for _ in range(1, hdu):
            hx, _ = _read_header(f)
            _skip_data(f, hx)
        hx, order = _read_header(f)
        if str(hx.get("XTENSION", "")).strip() != "BINTABLE":
            raise ValueError("HDU %d is not a binary table" % hdu)
        nrows, rowlen = int(hx["NAXIS2"]), int(hx["NAXIS1"])
        dt = _column_dtype(hx)
        if dt.itemsize != rowlen:
            raise ValueError("FITS row length %d does not match TFORMs (%d)" % (rowlen, dt.itemsize))
        raw = f.read(nrows * rowlen)
        if len(raw) < nrows * rowlen:
            raise ValueError("truncated FITS data")
    if str(hx.get("INDXSCHM", "IMPLICIT")).strip().upper() != "IMPLICIT":
        raise NotImplementedError("partial-sky (EXPLICIT) HEALPix maps are not supported")
    table = np.frombuffer(raw, dtype=dt, count=nrows)
    fields = (field,) if isinstance(field, (int, np.integer)) else tuple(field)
    ordering = str(hx.get("ORDERING", "RING")).strip().upper()
    maps = []
    for fi in fields:
        k = int(fi) + 1
        rawcol = table["c%d" % k].reshape(-1)
        col = rawcol.astype(np.float64) * float(hx.get("TSCAL%d" % k, 1.0)) + float(hx.get("TZERO%d" % k, 0.0))
        if "TNULL%d" % k in hx:
            col[rawcol == hx["TNULL%d" % k]] = UNSEEN
        nside = npix2nside(col.size)
        if "NSIDE" in hx and int(hx["NSIDE"]) != nside:
            raise ValueError("NSIDE keyword %s does not match the map size" % hx["NSIDE"])
        if ordering.startswith("NEST") and not nest:
            col = reorder(col, n2r=True)
        elif ordering == "RING" and nest:
            col = reorder(col, r2n=True)
        maps.append(col.astype(dtype, copy=False))
    out = maps[0] if len(maps) == 1 else np.stack(maps)
    return (out, [(key, hx[key]) for key in order]) if h else out


def _card(key, value):
    if isinstance(value, bool):
        v = "%20s" % ("T" if value else "F")
    elif isinstance(value, (int, np.integer)):
        v = "%20d" % value
    elif isinstance(value, float):
        v = "%20s" % repr(value).upper()
    else:
        v = "'%-8s'" % str(value).replace("'", "''")
    return ("%-8s= %s" % (key, v))[:80].ljust(80)


def _header_bytes(cards):
    txt = "".join(cards) + "END".ljust(80)
    return txt.ljust((len(txt) + _BLOCK - 1) // _BLOCK * _BLOCK).encode("ascii")


def write_map(filename, m, nest=False, dtype=np.float32, column_names=None, overwrite=False, coord=None):
    """healpy.write_map for one or more full-sky maps (IMPLICIT binary table,
    1024 pixels per row when the map size allows)."""
    if os.path.exists(filename) and not overwrite:
        raise OSError("file exists: %s" % filename)
    maps = np.atleast_2d(np.asarray(m))
    npix = maps.shape[1]
    nside = npix2nside(npix)
    code = {np.dtype(np.float32): "E", np.dtype(np.float64): "D", np.dtype(np.int32): "J",
            np.dtype(np.int64): "K", np.dtype(np.int16): "I", np.dtype(np.uint8): "B"}[np.dtype(dtype)]
    rep = 1024 if npix % 1024 == 0 else 1
    nrows = npix // rep
    names = column_names or (["TEMPERATURE", "Q_POLARISATION", "U_POLARISATION"][:len(maps)]
                             if len(maps) <= 3 else ["MAP%d" % i for i in range(len(maps))])
    dt = np.dtype([("c%d" % k, _TFORM[code], (rep,)) for k in range(len(maps))])
    table = np.empty(nrows, dtype=dt)
    for k in range(len(maps)):
        table["c%d" % k] = maps[k].astype(dtype).reshape(nrows, rep)
    prim = _header_bytes([_card("SIMPLE", True), _card("BITPIX", 8), _card("NAXIS", 0), _card("EXTEND", True)])
    cards = [_card("XTENSION", "BINTABLE"), _card("BITPIX", 8), _card("NAXIS", 2), _card("NAXIS1", dt.itemsize),
             _card("NAXIS2", nrows), _card("PCOUNT", 0), _card("GCOUNT", 1), _card("TFIELDS", len(maps))]
    for k in range(len(maps)):
        cards += [_card("TTYPE%d" % (k + 1), names[k]), _card("TFORM%d" % (k + 1), "%d%s" % (rep, code))]
    cards += [_card("PIXTYPE", "HEALPIX"), _card("ORDERING", "NESTED" if nest else "RING"), _card("NSIDE", nside),
              _card("FIRSTPIX", 0), _card("LASTPIX", npix - 1), _card("INDXSCHM", "IMPLICIT"),
              _card("OBJECT", "FULLSKY")]
    if coord:
        cards.append(_card("COORDSYS", coord))
    data = table.tobytes()
    with open(filename, "wb") as f:
        f.write(prim)
        f.write(_header_bytes(cards))
        f.write(data + b"\0" * ((-len(data)) % _BLOCK))


# ---------------------------------------------------------------------------------------
# run / dataset records (main_polarization.py)
# ---------------------------------------------------------------------------------------
def run_record(h_cls, h_accept_cr, h_duration_cr, bins, blocks, proposal_variances, total_time, total_cpu_time,
               pcg_accuracy=None, rj_step=False, gibbs_iterations=None, gibbs_cr=False, h_accept_nc=None,
               h_duration_cls_centered=None, h_duration_cls_non_centered=None, h_duration_iteration=None):
    """the dict main_polarization.py:172-181 builds (same keys; the reference
    stores h_accept_cr under both h_accept_nc and h_accept_cr)."""
    return {"h_cls": h_cls, "h_accept_nc": h_accept_cr if h_accept_nc is None else h_accept_nc,
            "h_duration_cls_centered": h_duration_cls_centered, "h_duration_cr": h_duration_cr,
            "bins_EE": bins["EE"], "bins_BB": bins["BB"], "blocks_EE": blocks["EE"],
            "h_duration_cls_non_centered": h_duration_cls_non_centered,
            "h_duration_iteration": h_duration_iteration, "blocks_BB": blocks["BB"],
            "proposal_variances_EE": proposal_variances["EE"], "proposal_variances_BB": proposal_variances["BB"],
            "total_cpu_time": total_cpu_time, "pcg_accuracy": pcg_accuracy, "h_accept_cr": h_accept_cr,
            "total_time": total_time, "rj_step": rj_step, "gibbs_iterations": gibbs_iterations,
            "gibbs_cr": gibbs_cr}


def dataset_record(pix_map, skymap_true, cls_, fwhm_beam, noise_var_temp, noise_var_pol, mask_path, nside, lmax,
                   params_=None):
    """the dataset dict of main_polarization.py:77-81."""
    return {"pix_map": pix_map, "params_": params_, "skymap_true": skymap_true, "cls_": cls_,
            "fwhm_arcmin_beam": fwhm_beam, "noise_var_temp": noise_var_temp, "noise_var_pol": noise_var_pol,
            "mask_path": mask_path, "NSIDE": nside, "lmax": lmax}


def _flatten(d, prefix, out, kinds):
    for k, v in d.items():
        key = prefix + k
        if isinstance(v, dict):
            kinds[key] = "dict"
            _flatten(v, key + "/", out, kinds)
        elif v is None:
            kinds[key] = "none"
        elif isinstance(v, str):
            kinds[key] = "str"
            out[key] = np.array(v)
        else:
            a = np.asarray(v)
            if a.dtype == object:
                raise TypeError("save_npz: %s is not a plain array" % key)
            kinds[key] = "array"
            out[key] = a


def save_npz(path, record):
    """write a (nested) dict of arrays / scalars / strings / None as a plain
    .npz (no pickling; nested keys joined with '/')."""
    out, kinds = {}, {}
    _flatten(record, "", out, kinds)
    out["__kinds__"] = np.array([k + "\t" + v for k, v in kinds.items()])
    np.savez(path, **out)


def load_npz(path):
    """inverse of save_npz (allow_pickle stays False)."""
    with np.load(path, allow_pickle=False) as z:
        kinds = dict(s.split("\t", 1) for s in z["__kinds__"].tolist())
        rec = {}
        for key, kind in kinds.items():
            parts = key.split("/")
            node = rec
            for p in parts[:-1]:
                node = node.setdefault(p, {})
            if kind == "dict":
                node.setdefault(parts[-1], {})
            elif kind == "none":
                node[parts[-1]] = None
            elif kind == "str":
                node[parts[-1]] = str(z[key])
            else:
                a = z[key]
                node[parts[-1]] = a.item() if a.ndim == 0 else a
    return rec
