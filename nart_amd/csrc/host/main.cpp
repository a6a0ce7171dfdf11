// `nart <scene file> <output path> [-w -h -b -s -o -f -r] [--gpus N | --devices a,b,...] [--device d]`
// -- drop-in for the reference CLI (src/core/main.cpp:12-61) with RenderSession::Render() served
// by the MI355X path.  The reference's flags are parsed by nart_parse_args exactly as
// ParseRenderParamArguments does (render.cpp:236-325); the device flags are this build's own and
// are taken out of argv first:
//   --gpus N        render every session over GPUs 0..N-1 (or d..d+N-1 with --device d); "all" = every
//                   visible GPU.  Buckets are sharded over the GPUs and gathered with RCCL
//                   (nart_hip_create_multi); the image is bit-identical for any N.
//   --devices a,b   an explicit device list (repeats allowed: a rehearsal on fewer GPUs)
//   --device d      first (or only) device; NART_DEVICE sets the default, which is 0
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../../include/nart_hip.h"

namespace {

bool parse_int(const char* s, int& v) {
    char* end = nullptr;
    long x = std::strtol(s, &end, 10);
    if (!s[0] || *end) return false;
    v = (int)x;
    return true;
}

// Removes the device flags from argv (kept: everything the reference CLI parses).
bool take_device_flags(std::vector<char*>& args, std::vector<int>& devices) {
    int first = 0, gpus = 1;
    bool all = false;
    if (const char* e = std::getenv("NART_DEVICE")) parse_int(e, first);
    std::vector<int> list;
    std::vector<char*> kept;
    for (size_t i = 0; i < args.size(); ++i) {
        const char* a = args[i];
        const bool dev = !std::strcmp(a, "--device"), g = !std::strcmp(a, "--gpus"), l = !std::strcmp(a, "--devices");
        if (!dev && !g && !l) {
            kept.push_back(args[i]);
            continue;
        }
        if (i + 1 >= args.size()) {
            std::fprintf(stderr, "Error: %s needs a value\n", a);
            return false;
        }
        const char* v = args[++i];
        if (dev && !parse_int(v, first)) {
            std::fprintf(stderr, "Error: --device %s\n", v);
            return false;
        }
        if (g) {
            if (!std::strcmp(v, "all")) all = true;
            else if (!parse_int(v, gpus) || gpus < 1) {
                std::fprintf(stderr, "Error: --gpus %s\n", v);
                return false;
            }
        }
        if (l) {
            std::string s(v);
            size_t pos = 0;
            while (pos <= s.size()) {
                size_t c = s.find(',', pos);
                if (c == std::string::npos) c = s.size();
                int d = 0;
                if (!parse_int(s.substr(pos, c - pos).c_str(), d)) {
                    std::fprintf(stderr, "Error: --devices %s\n", v);
                    return false;
                }
                list.push_back(d);
                pos = c + 1;
            }
        }
    }
    args = kept;
    if (!list.empty()) {
        devices = list;
        return true;
    }
    if (all) {
        int n = 0;
        if (nart_hip_device_count(&n) != NART_OK || n < 1) {
            std::fprintf(stderr, "Error: no HIP devices\n");
            return false;
        }
        gpus = n - first;
    }
    for (int d = 0; d < gpus; ++d) devices.push_back(first + d);
    return true;
}

}  // namespace

int main(int argc, char* argv[]) {
    std::vector<char*> args(argv, argv + argc);
    std::vector<int> devices;
    if (!take_device_flags(args, devices)) return EXIT_FAILURE;
    if (args.size() < 3) {
        std::fprintf(stderr, "Too few arguments given.\nUsage example: %s <scene file> <output path>\n", argv[0]);
        return EXIT_FAILURE;
    }
    nart_render_params params;
    nart_render_params_init(&params);
    if (nart_parse_args((int)args.size(), args.data(), &params) != NART_OK) {
        std::fprintf(stderr, "%s\n", nart_scene_last_error());
        return EXIT_FAILURE;
    }
    std::printf("Loading %s...\n", args[1]);
    nart_scene* scene = nullptr;
    if (nart_scene_load(args[1], &scene) != NART_OK) {
        std::fprintf(stderr, "%s\nAborting.\n", nart_scene_last_error());
        return EXIT_FAILURE;
    }
    int n = nart_load_sessions(args[1], &params, nullptr, 0);
    if (n <= 0) {
        std::fprintf(stderr, "Failed to load sessions from %s\n", args[1]);
        return EXIT_FAILURE;
    }
    std::vector<nart_render_params> sessions(n);
    nart_load_sessions(args[1], &params, sessions.data(), n);
    nart_ctx* ctx = nullptr;
    int rc = nart_hip_create_multi(nart_scene_blob_of(scene), devices.data(), (int)devices.size(), &ctx);
    if (rc != NART_OK) {
        std::fprintf(stderr, "Error: cannot create the HIP render context on %zu device(s) (%d)\n", devices.size(), rc);
        return EXIT_FAILURE;
    }
    int k = 0;
    for (const nart_render_params& p : sessions) {
        auto start = std::chrono::high_resolution_clock::now();
        std::printf("Rendering...\n");
        nart_session_geometry g;
        nart_session_geometry_of(&p, &g);
        std::vector<nart_pixel> image((size_t)g.total_width * g.total_height);
        rc = nart_hip_render(ctx, &p, image.data(), nullptr);
        if (rc != NART_OK) {
            std::fprintf(stderr, "Error: render failed (%d): %s\n", rc, nart_hip_last_error(ctx));
            return EXIT_FAILURE;
        }
        // main.cpp:44-49: <out>.exr for one session, <out>_<n>.exr for several
        std::string path = std::string(args[2]) + (n == 1 ? std::string(".exr") : "_" + std::to_string(k++) + ".exr");
        std::printf("Writing to %s...\n", path.c_str());
        if (nart_write_exr(path.c_str(), &p, image.data(), 3) != NART_OK) {
            std::fprintf(stderr, "%s\n", nart_scene_last_error());
            return EXIT_FAILURE;
        }
        std::chrono::duration<float> d = std::chrono::high_resolution_clock::now() - start;
        std::printf("Completed in %gs\n", d.count());
        std::fflush(stdout);
    }
    nart_hip_destroy(ctx);
    nart_scene_free(scene);
    return 0;
}
