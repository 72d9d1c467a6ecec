/* grk_plugin_abi.h -- Grok's plugin ABI (minpf), as exported by
 * libgrok_plugin.so (grokimagecompression_amd/lib/), SURVEY.md §8(b2).
 *
 * Grok's host (`grk_plugin_load`, grok.cpp:834-861) dlopens
 * <plugin_path>/libgrok_plugin.so, calls minpf_post_load_plugin (which must
 * register one object, version {1, 0}; minpf_plugin.h:37-57, stub
 * src/lib/jp2_plugin/Plugin.cpp:32-50) and then dlsyms the plugin_* functions
 * by name (grok.cpp:810-823; typedefs plugin_interface.h:46-130).
 *
 * This plugin runs on the MI355X library (grk_mi355x.h):
 *   plugin_init            -> grkgpu_create(deviceId): true iff a gfx950 GPU
 *                             context is up (false: the host stays on its CPU path)
 *   plugin_get_debug_state -> GRK_PLUGIN_STATE_NO_DEBUG
 *   plugin_encode / plugin_batch_encode / plugin_decode /
 *   plugin_init_batch_decode / plugin_batch_decode
 *                          -> -1 ("not handled": the host codes the tile itself,
 *                             plugin_interface.h return convention).  The
 *                             per-tile hand-off needs Grok's grk_cparameters /
 *                             grk_image layouts, which this ABI does not
 *                             re-declare; the MI355X path is reached through
 *                             grk_mi355x.h instead.
 * Types that cross this boundary are re-declared here with the same layout
 * as the reference's; the others are opaque pointers.
 */
#ifndef GRK_PLUGIN_ABI_H
#define GRK_PLUGIN_ABI_H

#include <stdbool.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* minpf_plugin.h:22-57 */
struct minpf_platform_services;
typedef struct minpf_object_params {
    const char *id;
    const struct minpf_platform_services *platformServices;
} minpf_object_params;
typedef struct minpf_plugin_api_version {
    int32_t major;
    int32_t minor;
} minpf_plugin_api_version;
typedef void *(*minpf_create_func)(minpf_object_params *);
typedef int32_t (*minpf_destroy_func)(void *);
typedef struct minpf_register_params {
    minpf_plugin_api_version version;
    minpf_create_func createFunc;
    minpf_destroy_func destroyFunc;
} minpf_register_params;
typedef int32_t (*minpf_register_func)(const char *nodeType, const minpf_register_params *params);
typedef int32_t (*minpf_invoke_service_func)(const char *serviceName, void *serviceParams);
typedef struct minpf_platform_services {
    minpf_plugin_api_version version;
    minpf_register_func registerObject;
    minpf_invoke_service_func invokeService;
} minpf_platform_services;
typedef int32_t (*minpf_exit_func)(void);

/* grok.h:1816-1819 */
typedef struct grk_plugin_init_info {
    int32_t deviceId;
    bool verbose;
} grk_plugin_init_info;

#define GRK_PLUGIN_STATE_NO_DEBUG 0x0 /* grok.h:1791 */

/* Object id registered with the host (the reference stub uses "SamplePlugin",
 * Plugin.cpp:17). */
#define GRKGPU_PLUGIN_ID "GrokMI355X"

minpf_exit_func minpf_post_load_plugin(const char *pluginPath, const minpf_platform_services *services);
bool plugin_init(grk_plugin_init_info info);
uint32_t plugin_get_debug_state(void);
int32_t plugin_encode(void *encode_parameters, void *user_callback);
int32_t plugin_batch_encode(const char *input_dir, const char *output_dir, void *encode_parameters,
                            void *user_callback);
bool plugin_is_batch_complete(void);
void plugin_stop_batch_encode(void);
int32_t plugin_decode(void *decode_parameters, void *user_callback);
int32_t plugin_init_batch_decode(const char *input_dir, const char *output_dir, void *decode_parameters,
                                 void *user_callback);
int32_t plugin_batch_decode(void);
void plugin_stop_batch_decode(void);
/* debug hooks (plugin_interface.h:44-45; the stub's name for the first is
 * plugin_debug_next_cxd, Plugin.cpp:121 -- both names are exported) */
void plugin_debug_mqc_next_cxd(void *mqc, uint32_t d);
void plugin_debug_next_cxd(void *mqc, uint32_t d);
void plugin_debug_mqc_next_plane(void *mqc);

#ifdef __cplusplus
}
#endif
#endif
