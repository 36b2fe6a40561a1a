"""C-ABI checks that need no GPU: the library loads, exports every symbol include/ptgs/*.h declares,
struct layouts match the reference's (GeneralHeaders.h), and compute entry
points fail loudly (no CPU fallback) when there is no device."""
import ctypes as C
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADERS = [os.path.join(ROOT, "include", "ptgs", f) for f in ("ptgs.h", "ptgs_host.h")]


def _declared_functions():
    names = set()
    for h in HEADERS:
        text = open(h).read()
        text = re.sub(r"/\*.*?\*/", "", text, flags=re.S)
        for m in re.finditer(r"\b(ptgs_[a-z0-9_]+)\s*\(", text):
            names.add(m.group(1))
    return names


def test_every_declared_symbol_is_exported(native_lib):
    from pathtracer_gaussiansplatting_amd import _abi
    declared = _declared_functions()
    assert len(declared) >= 30
    for name in sorted(declared):
        assert hasattr(native_lib, name), f"{name} declared in include/ptgs but not exported"
    # the Python mirror binds every declared symbol with a signature
    assert declared == set(_abi.SYMBOLS), declared ^ set(_abi.SYMBOLS)


def test_abi_version_and_arch(native_lib):
    assert native_lib.ptgs_abi_version() == 4  # 4: PTGS_EBADIDS, PTGS_FLAG_SPLAT_OVERLAP (3: ids / fused / spill fields)
    assert native_lib.ptgs_device_arch() == b"gfx950"


def test_struct_layouts():
    from pathtracer_gaussiansplatting_amd import _abi
    # ptgs_splat_status (ABI 3): frames u64, views[8], 4 x u32, spilled / incomplete tiles u64, 2 x u32
    st = _abi.SplatStatus
    assert C.sizeof(st) == 80 and st.spilled_tiles.offset == 56 and st.spill_demand.offset == 76
    # Appendix B sizes / offsets
    assert _abi.VERTEX_DTYPE.itemsize == 80
    assert _abi.VERTEX_DTYPE.fields["normal"][1] == 16 and _abi.VERTEX_DTYPE.fields["tex_coord"][1] == 64
    m = _abi.MATERIAL_DTYPE
    assert m.itemsize == 308
    assert m.fields["emissive_factor_and_pad"][1] == 208 and m.fields["metallic_factor"][1] == 224
    assert m.fields["transmission_factor"][1] == 256 and m.fields["pad"][1] == 268
    assert m.fields["albedo_texture_index"][1] == 272 and m.fields["sg_id"][1] == 300
    assert m.fields["use_specular_glossiness_workflow"][1] == 304
    assert C.sizeof(_abi.Ubo) == 192 and _abi.Ubo.frame_count.offset == 140 and _abi.Ubo.ambient_light.offset == 144
    assert _abi.Ubo.emissive_flux.offset == 160 and _abi.Ubo.fov.offset == 176
    assert _abi.PUNCTUAL_LIGHT_DTYPE.itemsize == 64 and _abi.PUNCTUAL_LIGHT_DTYPE.fields["type"][1] == 52
    for dt in (_abi.MESH_INFO_DTYPE, _abi.LIGHT_TRIANGLE_DTYPE, _abi.LIGHT_CDF_DTYPE, _abi.PUNCTUAL_CDF_DTYPE):
        assert dt.itemsize == 16
    assert _abi.HITDATA_DTYPE.itemsize == 48 and _abi.HITDATA_DTYPE.fields["flag"][1] == 12
    assert _abi.HITDATA_DTYPE.fields["normal"][1] == 32
    assert C.sizeof(_abi.RayPush) == 80 and _abi.RayPush.mode.offset == 64 and _abi.RayPush.height.offset == 76
    # ptgs.h (ABI 2): ptgs_texture and the texture table at the end of ptgs_scene_desc
    assert C.sizeof(_abi.Texture) == 24 and _abi.Texture.srgb.offset == 16
    assert _abi.SceneDesc.textures.offset == _abi.SceneDesc.blue_noise_size.offset + 8
    assert _abi.SceneDesc.num_textures.offset == _abi.SceneDesc.textures.offset + 8


def test_compute_path_fails_loudly_without_gpu(native_lib):
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    h = C.c_void_p()
    rc = native_lib.ptgs_create(0, C.byref(h))
    assert rc == -2 and not h.value  # PTGS_EHIP: no device, no silent CPU path
    from pathtracer_gaussiansplatting_amd import PtgsError, Renderer
    with pytest.raises(PtgsError):
        Renderer(0)


def test_null_arguments_rejected(native_lib):
    assert native_lib.ptgs_create(0, None) == -1
    assert native_lib.ptgs_scene_upload(None, None) == -1
    assert native_lib.ptgs_trace_camera(None, None, 1, 1, None, 1, 1, 0, None) == -1
    assert native_lib.ptgs_mat4_inverse(None, None) == -1
    z = np.zeros(16, np.float32)
    out = np.zeros(16, np.float32)
    from pathtracer_gaussiansplatting_amd._abi import fptr
    assert native_lib.ptgs_mat4_inverse(fptr(z), fptr(out)) == -1  # singular


def test_missing_library_fails_loudly(tmp_path):
    from pathtracer_gaussiansplatting_amd import _abi
    with pytest.raises(_abi.PtgsError):
        _abi.load_library(str(tmp_path / "libptgs.so"))


def test_rccl_unique_id_without_gpu(native_lib):
    """The RCCL bootstrap id needs no device: the C-ABI resolves librccl at run time."""
    buf = (C.c_uint8 * 128)()
    assert native_lib.ptgs_comm_unique_id(buf) == 0
    assert any(bytes(buf))
    assert native_lib.ptgs_comm_unique_id(None) == -1  # PTGS_EINVAL


def _compile_layout(include_dir, cxx=False):
    import subprocess
    src = os.path.join(ROOT, "tests", "native", "abi_layout.c")
    cmd = (["g++", "-std=c++17", "-x", "c++"] if cxx else ["gcc", "-std=c11", "-pedantic-errors"])
    cmd += ["-Wall", "-Werror", "-fsyntax-only", "-I", include_dir, src]
    return subprocess.run(cmd, capture_output=True, text=True)


def test_header_layouts_compile_in_c_and_cxx():
    """include/ptgs/ptgs.h's static layout asserts (GeneralHeaders.h sizes / offsets) hold as C11 and C++."""
    inc = os.path.join(ROOT, "include")
    for cxx in (False, True):
        r = _compile_layout(inc, cxx)
        assert r.returncode == 0, r.stderr


@pytest.mark.parametrize("old,new", [("float pad1;", "float pad1, extra;"),
                                     ("int32_t sg_id;", "int64_t sg_id;"),
                                     ("uint32_t frame_count;", "uint64_t frame_count;")])
def test_header_layout_drift_fails_to_compile(tmp_path, old, new):
    """A drifted copy of the header (one field changed) must not compile: the asserts are live."""
    text = open(HEADERS[0]).read()
    assert old in text
    (tmp_path / "ptgs").mkdir()
    (tmp_path / "ptgs" / "ptgs.h").write_text(text.replace(old, new, 1))
    r = _compile_layout(str(tmp_path))
    assert r.returncode != 0 and "static assert" in r.stderr.lower(), r.stderr
