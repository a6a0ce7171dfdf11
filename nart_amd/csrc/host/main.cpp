// `nart <scene file> <output path> [-w -h -b -s -o -f -r]` -- drop-in for the reference CLI
// (src/core/main.cpp:12-61) with RenderSession::Render() served by the MI355X path.
// The device ordinal comes from NART_DEVICE (default 0) so the flag surface stays identical.
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <string>
#include <vector>

#include "../../../include/nart_hip.h"

int main(int argc, char* argv[]) {
    if (argc < 3) {
        std::fprintf(stderr, "Too few arguments given.\nUsage example: %s <scene file> <output path>\n", argv[0]);
        return EXIT_FAILURE;
    }
    nart_render_params params;
    nart_render_params_init(&params);
    if (nart_parse_args(argc, argv, &params) != NART_OK) {
        std::fprintf(stderr, "%s\n", nart_scene_last_error());
        return EXIT_FAILURE;
    }
    std::printf("Loading %s...\n", argv[1]);
    nart_scene* scene = nullptr;
    if (nart_scene_load(argv[1], &scene) != NART_OK) {
        std::fprintf(stderr, "%s\nAborting.\n", nart_scene_last_error());
        return EXIT_FAILURE;
    }
    int n = nart_load_sessions(argv[1], &params, nullptr, 0);
    if (n <= 0) {
        std::fprintf(stderr, "Failed to load sessions from %s\n", argv[1]);
        return EXIT_FAILURE;
    }
    std::vector<nart_render_params> sessions(n);
    nart_load_sessions(argv[1], &params, sessions.data(), n);
    const char* dev = std::getenv("NART_DEVICE");
    nart_ctx* ctx = nullptr;
    int rc = nart_hip_create(nart_scene_blob_of(scene), dev ? std::atoi(dev) : 0, &ctx);
    if (rc != NART_OK) {
        std::fprintf(stderr, "Error: cannot create the HIP render context (%d)\n", rc);
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
        std::string path = std::string(argv[2]) + (n == 1 ? std::string(".exr") : "_" + std::to_string(k++) + ".exr");
        std::printf("Writing to %s...\n", path.c_str());
        if (nart_write_exr(path.c_str(), &p, image.data(), 3) != NART_OK) {
            std::fprintf(stderr, "%s\n", nart_scene_last_error());
            return EXIT_FAILURE;
        }
        std::chrono::duration<float> d = std::chrono::high_resolution_clock::now() - start;
        std::printf("Completed in %gs\n", d.count());
    }
    nart_hip_destroy(ctx);
    nart_scene_free(scene);
    return 0;
}
