// libgrok_plugin.so: Grok's minpf plugin ABI on top of libgrk_mi355x.so
// (include/grk_plugin_abi.h).  Host side: grok.cpp:810-861.
#include "../../include/grk_plugin_abi.h"
#include "../../include/grk_mi355x.h"

#include <mutex>

#define PLUGIN_API __attribute__((visibility("default")))

namespace {
std::mutex g_mu;
grkgpu_ctx *g_ctx = nullptr;  // one GPU context per loaded plugin (grok's plugin manager is a global too)

int32_t exit_plugin(void) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx) grkgpu_destroy(g_ctx);
    g_ctx = nullptr;
    return 0;
}
// minpf object factory: Grok never calls these for the T1 plugin (Plugin.cpp:24-31)
void *create_object(minpf_object_params *) { return nullptr; }
int32_t destroy_object(void *) { return 0; }
}  // namespace

extern "C" {

PLUGIN_API minpf_exit_func minpf_post_load_plugin(const char *, const minpf_platform_services *services) {
    if (!services || !services->registerObject) return nullptr;
    minpf_register_params rp;
    rp.version.major = 1;
    rp.version.minor = 0;
    rp.createFunc = create_object;
    rp.destroyFunc = destroy_object;
    if (services->registerObject(GRKGPU_PLUGIN_ID, &rp) < 0) return nullptr;
    return exit_plugin;
}

// grk_plugin_init (grok.cpp:877-890): false keeps the host on its CPU path.
PLUGIN_API bool plugin_init(grk_plugin_init_info info) {
    std::lock_guard<std::mutex> lk(g_mu);
    if (g_ctx) return true;
    return grkgpu_create(info.deviceId < 0 ? 0 : info.deviceId, &g_ctx) == GRKGPU_OK;
}

PLUGIN_API uint32_t plugin_get_debug_state(void) { return GRK_PLUGIN_STATE_NO_DEBUG; }

// -1 = not handled: the host codes the tile on its own path (plugin_interface.h)
PLUGIN_API int32_t plugin_encode(void *, void *) { return -1; }
PLUGIN_API int32_t plugin_batch_encode(const char *, const char *, void *, void *) { return -1; }
PLUGIN_API bool plugin_is_batch_complete(void) { return true; }
PLUGIN_API void plugin_stop_batch_encode(void) {}
PLUGIN_API int32_t plugin_decode(void *, void *) { return -1; }
PLUGIN_API int32_t plugin_init_batch_decode(const char *, const char *, void *, void *) { return -1; }
PLUGIN_API int32_t plugin_batch_decode(void) { return -1; }
PLUGIN_API void plugin_stop_batch_decode(void) {}
PLUGIN_API void plugin_debug_mqc_next_cxd(void *, uint32_t) {}
PLUGIN_API void plugin_debug_next_cxd(void *, uint32_t) {}
PLUGIN_API void plugin_debug_mqc_next_plane(void *) {}

}  // extern "C"
