"""Quick GPU timing of the render path (development aid, not the bench contract)."""
import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)

import nart_amd  # noqa: E402
from nart_amd import scenes  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scene", default="glass")
    ap.add_argument("-w", type=int, default=1920)
    ap.add_argument("-H", type=int, default=1080)
    ap.add_argument("-s", type=int, default=16)
    ap.add_argument("--counters", action="store_true")
    ap.add_argument("--spec", type=int, default=2, help="path-kernel builds: 0 generic, 1 specialised, 2 + lean")
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--bounces", type=int, default=0, help="override the scene's bounce limit")
    ap.add_argument("--env", type=int, default=1024, help="c4: environment map width (height = width / 2)")
    ap.add_argument("--flat", default="", help="c4 diagnostics: comma list of rho_d,roughness,normal to replace "
                                               "by constants (not a parity configuration)")
    a = ap.parse_args()
    if a.scene == "c4":
        path = scenes.c4_teapot(env_size=(a.env, a.env // 2))
        if a.flat:
            js = json.load(open(path))
            mat = js["meshes"][1]["material"]
            for k in a.flat.split(","):
                if k == "normal":
                    mat.pop("normal")
                else:
                    mat[k] = [0.5, 0.4, 0.3] if k == "rho_d" else 0.3
            json.dump(js, open(path, "w"))
    elif a.scene == "c5":
        path = scenes.volume(width=a.w, height=a.H, spp=a.s, kind="c5")
    else:
        path = scenes.glass_sphere() if a.scene == "glass" else scenes.cornell()
    scene = nart_amd.Scene(path)
    p = nart_amd.load_sessions(path)[0]
    p.image_width, p.image_height, p.spp = a.w, a.H, a.s
    if a.bounces:
        p.bounces = a.bounces
    r = nart_amd.HipRenderer(scene)
    r.set_specialize(a.spec)
    for rep in range(a.reps):
        st = nart_amd.RenderStats()
        t = time.time()
        r.render(p, st)
        dt = time.time() - t
        d = st.as_dict()
        d["wall_s"] = dt
        d["msamples_per_s_kernel"] = d["samples"] / (d["kernel_ms"] * 1e3)
        d["msamples_per_s_wall"] = d["samples"] / dt / 1e6
        d["features"], d["build"] = r.scene_features()
        print(json.dumps(d), flush=True)
    if a.counters:
        r.set_counters(True)
        st = nart_amd.RenderStats()
        r.render(p, st)
        d = st.as_dict()
        n = d["traced_samples"]
        d.update({k + "_per_sample": d[k] / n for k in ("rays_extend", "rays_shadow", "node_visits", "tri_tests",
                                                          "bounces")})
        print(json.dumps(d), flush=True)


if __name__ == "__main__":
    main()
