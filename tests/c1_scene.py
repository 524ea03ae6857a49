"""The C1 test scene (models/teapot/scene.xml:1-84 structure) written into a directory: the scene
XML, the seeded stand-in meshes of teapot_meshes.py and a synthetic sky as PFM.  Shared by
tests/test_c1_mesh_host.py (CPU: loading, BVH, refusals) and tests/test_gpu_c1.py (device parity).
The reference's own scene file and envmap are not used, so the tests run where /root/reference is
absent (the GPU box)."""
import os

import numpy as np

import teapot_meshes

SCENE = """<?xml version="1.0" encoding="utf-8"?>
<scene version="0.6.0">
  <default name="w" value="64"/>
  <default name="h" value="64"/>
  <default name="spp" value="16"/>
  <integrator type="path">
    <integer name="maxDepth" value="65"/>
    <boolean name="strictNormals" value="true"/>
  </integrator>
  <sensor type="perspective">
    <float name="fov" value="35"/>
    <transform name="toWorld">
      <matrix value="-0.00550949 -0.342144 -0.939631 23.895 1.07844e-005 0.939646 -0.342149 11.2207 0.999985 -0.00189103 -0.00519335 0.0400773 0 0 0 1"/>
    </transform>
    <sampler type="sobol"><integer name="sampleCount" value="$spp"/></sampler>
    <film type="ldrfilm">
      <integer name="width" value="$w"/>
      <integer name="height" value="$h"/>
      <float name="gamma" value="2.2"/>
      <boolean name="banner" value="false"/>
      <rfilter type="tent"/>
    </film>
  </sensor>
  <bsdf type="twosided" id="Material">
    <bsdf type="plastic">
      <float name="intIOR" value="1.5"/>
      <float name="extIOR" value="1"/>
      <boolean name="nonlinear" value="true"/>
      <rgb name="diffuseReflectance" value="0.9, 0.9, 0.9"/>
    </bsdf>
  </bsdf>
  <bsdf type="twosided" id="Floor">
    <bsdf type="diffuse">
      <texture name="reflectance" type="checkerboard">
        <rgb name="color1" value="0.325, 0.31, 0.25"/>
        <rgb name="color0" value="0.725, 0.71, 0.68"/>
        <float name="uoffset" value="0"/>
        <float name="voffset" value="0"/>
        <float name="uscale" value="10"/>
        <float name="vscale" value="10"/>
      </texture>
    </bsdf>
  </bsdf>
  <shape type="rectangle">
    <transform name="toWorld">
      <matrix value="-39.9766 39.9766 -1.74743e-006 0 4.94249e-006 2.47125e-006 -56.5355 0 -39.9766 -39.9766 -5.2423e-006 0 0 0 0 1"/>
    </transform>
    <ref id="Floor"/>
  </shape>
  <shape type="obj">
    <string name="filename" value="models/Mesh001.obj"/>
    <ref id="Material"/>
  </shape>
  <shape type="obj">
    <string name="filename" value="models/Mesh000.obj"/>
    <ref id="Material"/>
  </shape>
  <emitter type="envmap">
    <transform name="toWorld">
      <matrix value="-0.922278 0 0.386527 0 0 1 0 0 -0.386527 0 -0.922278 1.17369 0 0 0 1"/>
    </transform>
    <string name="filename" value="env.pfm"/>
  </emitter>
</scene>
"""


def synthetic_sky(w=128, h=64):
    """A smooth sky with a warm sun blob (linear RGB, top row first)."""
    y, x = np.mgrid[0:h, 0:w].astype(np.float64)
    theta = (y + 0.5) / h * np.pi
    phi = (x + 0.5) / w * 2 * np.pi
    base = np.clip(np.cos(theta), 0, None)[..., None] * np.array([0.35, 0.5, 0.9]) + 0.08
    d = np.stack([np.sin(theta) * np.sin(phi), np.cos(theta), -np.sin(theta) * np.cos(phi)], -1)
    sun = np.array([0.4, 0.75, 0.52])
    sun /= np.linalg.norm(sun)
    blob = np.exp(-(1 - d @ sun) * 60.0)[..., None] * np.array([40.0, 36.0, 30.0])
    return (base + blob).astype(np.float32)


def write_pfm(path, img):
    h, w, _ = img.shape
    with open(path, "wb") as f:
        f.write(b"PF\n%d %d\n-1.0\n" % (w, h))
        f.write(np.ascontiguousarray(img[::-1], "<f4").tobytes())



def variant_scene():
    """The other branches of the mesh path in the same scene: face normals on Mesh001
    (trimesh.cpp:608-616: no vertex normals, the geometric frame shades), flipped normals on the
    floor (rectangle.cpp:96-99) and on Mesh000 (vertex normals negated, trimesh.cpp:617-622), a
    one-sided linear plastic with a coloured specular on Mesh000 (no twosided wrapper: its back
    faces reflect nothing), a constant-reflectance diffuse floor, no strictNormals."""
    s = SCENE.replace('<boolean name="strictNormals" value="true"/>', '<boolean name="strictNormals" value="false"/>')
    s = s.replace("""  <bsdf type="twosided" id="Floor">""", """  <bsdf type="plastic" id="Knob">
    <float name="intIOR" value="1.33"/>
    <rgb name="diffuseReflectance" value="0.2, 0.5, 0.7"/>
    <rgb name="specularReflectance" value="0.8, 0.7, 0.6"/>
  </bsdf>
  <bsdf type="twosided" id="Floor">""")
    s = s.replace("""      <texture name="reflectance" type="checkerboard">
        <rgb name="color1" value="0.325, 0.31, 0.25"/>
        <rgb name="color0" value="0.725, 0.71, 0.68"/>
        <float name="uoffset" value="0"/>
        <float name="voffset" value="0"/>
        <float name="uscale" value="10"/>
        <float name="vscale" value="10"/>
      </texture>""", """      <rgb name="reflectance" value="0.6, 0.55, 0.5"/>""")
    s = s.replace("""    <ref id="Floor"/>""", """    <boolean name="flipNormals" value="true"/>
    <ref id="Floor"/>""")
    s = s.replace("""    <string name="filename" value="models/Mesh001.obj"/>""", """    <string name="filename" value="models/Mesh001.obj"/>
    <boolean name="faceNormals" value="true"/>""")
    s = s.replace("""    <string name="filename" value="models/Mesh000.obj"/>
    <ref id="Material"/>""", """    <string name="filename" value="models/Mesh000.obj"/>
    <boolean name="flipNormals" value="true"/>
    <ref id="Knob"/>""")
    assert s.count("flipNormals") == 2 and "faceNormals" in s and 'ref id="Knob"' in s
    return s


def write(d, variant=False):
    """Write the scene (or its variant_scene), its meshes and its sky under directory d; returns
    the scene path."""
    d = str(d)
    teapot_meshes.write_all(os.path.join(d, "models"))
    write_pfm(os.path.join(d, "env.pfm"), synthetic_sky())
    path = os.path.join(d, "scene_variant.xml" if variant else "scene.xml")
    with open(path, "w") as f:
        f.write(variant_scene() if variant else SCENE)
    return path
