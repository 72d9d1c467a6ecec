// Layout table of include/grk_plugin_abi.h's re-declarations.  Test infrastructure.
#include <stddef.h>
#include "../../include/grk_api.h"
#include "abi_fields.h"
using T_CPARAMS = grkp_cparameters;
using T_POC = grkp_poc;
using T_IMAGE = grkp_image;
using T_COMP = grkp_image_comp;
using T_CMPTPARM = grkp_image_cmptparm;
using T_PASS = grk_plugin_pass;
using T_CBLK = grk_plugin_code_block;
using T_PREC = grk_plugin_precinct;
using T_BAND = grk_plugin_band;
using T_RES = grk_plugin_resolution;
using T_TCOMP = grk_plugin_tile_component;
using T_TILE = grk_plugin_tile;
using T_INIT = grk_plugin_init_info;
using T_CBINFO = plugin_encode_user_callback_info;
using T_MINPF_REG = minpf_register_params;
using T_MINPF_SVC = minpf_platform_services;
using T_HINFO = grkp_header_info;
using T_DPARAMS = grkp_dparameters;
using T_DECOMP = grkp_decompress_parameters;
using T_DCBINFO = PluginDecodeCallbackInfo;
using T_TCCPINFO = grk_tccp_info;
using T_TILEINFO2 = grk_tile_info_v2;
using T_CSINFO = grk_codestream_info_v2;
using T_MARKER = grk_marker_info;
using T_TPIDX = grk_tp_index;
using T_PKTINFO = grk_packet_info;
using T_TILEIDX = grk_tile_index;
using T_CSIDX = grk_codestream_index;
extern const AbiEntry abi_ours[] = {ABI_FIELDS(ABI_EMIT_F, ABI_EMIT_S){nullptr, nullptr, 0}};
