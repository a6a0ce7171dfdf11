"""The one octree behaviour the device does not emulate (VERDICT r04 missing #4):
a triangle whose plane distance is NaN -- Triangle::Intersect's `t <= tMin || t >= tMax` lets NaN
through (geometry.cpp:37-39) and Chunk::Intersect then keeps scanning with isect.tMax = NaN
(bvh.cpp:66-79) -- when the BVH2 culled that triangle but it shares the winner's octree chunk.

t = (dot(v0, n) - dot(o, n)) / dot(d, n) is NaN only as 0/0: the numerator is exactly zero (the
ray origin lies on the triangle's plane in float arithmetic) AND dot(d, n) is exactly zero.  Every
camera ray of a session starts at the camera position, so for camera rays the first condition is
a property of the scene alone.  This test evaluates it, with the reference's float operations
(n = glm::cross(v1 - v0, v2 - v0), GLM's dot3 order), for every triangle of every scene the GPU
suite and the bench render: no triangle has zero area and no triangle plane contains the camera, so no camera ray can produce a
NaN plane distance in these scenes.  (Secondary rays start at biased hit points and would need
an exactly zero dot(d, n) as well, for a direction drawn from a continuous distribution; the
device already replays the octree for every NaN it does see -- octree.h.)"""
import numpy as np
import pytest

import nart_amd
from nart_amd import scenes


def _dot(a, b):
    return (a[..., 0] * b[..., 0] + a[..., 1] * b[..., 1]) + a[..., 2] * b[..., 2]


def _cross(a, b):
    return np.stack([a[..., 1] * b[..., 2] - b[..., 1] * a[..., 2],
                     a[..., 2] * b[..., 0] - b[..., 2] * a[..., 0],
                     a[..., 0] * b[..., 1] - b[..., 0] * a[..., 1]], axis=-1)


SCENES = {
    "glassSphere": lambda d: scenes.glass_sphere(d),
    "ring": lambda d: scenes.reference_scene("ring", d),
    "veach": lambda d: scenes.reference_scene("veach", d),
    "cornell": lambda d: scenes.cornell(d),
    "materials": lambda d: scenes.materials(d),
    "environment": lambda d: scenes.environment(d),
    "c4_teapot": lambda d: scenes.c4_teapot(d, env_size=(64, 32)),
}


@pytest.mark.parametrize("name", sorted(SCENES))
def test_no_triangle_plane_contains_the_camera(built, tmp_path, name):
    sc = nart_amd.Scene(SCENES[name](str(tmp_path)))
    t = sc.triangles().astype(np.float32)
    v0, v1, v2 = t[:, 0:3], t[:, 3:6], t[:, 6:9]
    n = _cross(v1 - v0, v2 - v0)
    _, m = sc.camera()
    # PinholeCamera::CastRay: o = vec4(0, 0, 0, 1) * cameraToWorld = (m[3], m[7], m[11])
    o = np.broadcast_to(np.float32([m[3], m[7], m[11]]), v0.shape)
    num = _dot(v0, n) - _dot(o, n)
    # a zero-area triangle (n == 0) would give 0/0 for every ray; none of these scenes has one
    assert not np.all(n == 0, axis=1).any(), name
    on_plane = num == 0
    assert not on_plane.any(), "%s: %d triangle planes contain the camera, e.g. %s" % (
        name, int(on_plane.sum()), np.nonzero(on_plane)[0][:5])
