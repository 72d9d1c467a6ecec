// oracle/abi/abi_fields.h -- the plugin-boundary fields whose layout
// include/grk_plugin_abi.h must share with the reference's grok.h /
// plugin_interface.h.  Each TU (abi_ref.cpp over the reference headers,
// abi_ours.cpp over ours) defines the T_* type names and expands this list
// into an offset table; abi_check compares the two.  Test infrastructure.
#define ABI_FIELDS(F, S)                                                                              \
    S(CPARAMS) F(CPARAMS, tile_size_on) F(CPARAMS, cp_tx0) F(CPARAMS, cp_tdx) F(CPARAMS, cp_disto_alloc) \
    F(CPARAMS, cp_fixed_quality) F(CPARAMS, cp_comment) F(CPARAMS, cp_comment_len)                    \
    F(CPARAMS, cp_is_binary_comment) F(CPARAMS, cp_num_comments) F(CPARAMS, csty) F(CPARAMS, prog_order) \
    F(CPARAMS, POC) F(CPARAMS, numpocs) F(CPARAMS, tcp_numlayers) F(CPARAMS, tcp_rates)                 \
    F(CPARAMS, tcp_distoratio) F(CPARAMS, numresolution) F(CPARAMS, cblockw_init) F(CPARAMS, cblockh_init) \
    F(CPARAMS, cblk_sty) F(CPARAMS, isHT) F(CPARAMS, irreversible) F(CPARAMS, roi_compno)              \
    F(CPARAMS, roi_shift) F(CPARAMS, res_spec) F(CPARAMS, prcw_init) F(CPARAMS, prch_init)             \
    F(CPARAMS, infile) F(CPARAMS, outfile) F(CPARAMS, image_offset_x0) F(CPARAMS, image_offset_y0)     \
    F(CPARAMS, subsampling_dx) F(CPARAMS, subsampling_dy) F(CPARAMS, decod_format) F(CPARAMS, cod_format) \
    F(CPARAMS, raw_cp) F(CPARAMS, max_comp_size) F(CPARAMS, tp_on) F(CPARAMS, tp_flag) F(CPARAMS, tcp_mct) \
    F(CPARAMS, mct_data) F(CPARAMS, max_cs_size) F(CPARAMS, rsiz) F(CPARAMS, framerate)                \
    F(CPARAMS, write_capture_resolution_from_file) F(CPARAMS, capture_resolution_from_file)           \
    F(CPARAMS, write_capture_resolution) F(CPARAMS, capture_resolution) F(CPARAMS, write_display_resolution) \
    F(CPARAMS, display_resolution) F(CPARAMS, rateControlAlgorithm) F(CPARAMS, numThreads)            \
    F(CPARAMS, deviceId) F(CPARAMS, duration) F(CPARAMS, kernelBuildOptions) F(CPARAMS, repeats)       \
    F(CPARAMS, verbose)                                                                               \
    S(POC) F(POC, resno0) F(POC, compno0) F(POC, layno1) F(POC, resno1) F(POC, compno1) F(POC, layno0) \
    F(POC, precno0) F(POC, precno1) F(POC, prg1) F(POC, prg) F(POC, progorder) F(POC, tile) F(POC, tx0) \
    F(POC, layS) F(POC, layE) F(POC, txS) F(POC, dx) F(POC, lay_t) F(POC, ty0_t)                      \
    S(IMAGE) F(IMAGE, x0) F(IMAGE, y1) F(IMAGE, numcomps) F(IMAGE, color_space) F(IMAGE, comps)         \
    F(IMAGE, icc_profile_buf) F(IMAGE, icc_profile_len) F(IMAGE, capture_resolution)                  \
    F(IMAGE, display_resolution) F(IMAGE, iptc_buf) F(IMAGE, iptc_len) F(IMAGE, xmp_buf) F(IMAGE, xmp_len) \
    S(COMP) F(COMP, dx) F(COMP, w) F(COMP, h) F(COMP, x0) F(COMP, prec) F(COMP, sgnd) F(COMP, resno_decoded) \
    F(COMP, data) F(COMP, owns_data) F(COMP, alpha)                                                   \
    S(CMPTPARM) F(CMPTPARM, dx) F(CMPTPARM, w) F(CMPTPARM, x0) F(CMPTPARM, prec) F(CMPTPARM, sgnd)     \
    S(PASS) F(PASS, distortionDecrease) F(PASS, rate) F(PASS, length)                                 \
    S(CBLK) F(CBLK, x0) F(CBLK, y1) F(CBLK, contextStream) F(CBLK, numPix) F(CBLK, compressedData)     \
    F(CBLK, compressedDataLength) F(CBLK, numBitPlanes) F(CBLK, numPasses) F(CBLK, passes) F(CBLK, sortedIndex) \
    S(PREC) F(PREC, numBlocks) F(PREC, blocks)                                                        \
    S(BAND) F(BAND, orient) F(BAND, numPrecincts) F(BAND, precincts) F(BAND, stepsize)                \
    S(RES) F(RES, level) F(RES, numBands) F(RES, bands)                                               \
    S(TCOMP) F(TCOMP, numResolutions) F(TCOMP, resolutions)                                           \
    S(TILE) F(TILE, decode_flags) F(TILE, numComponents) F(TILE, tileComponents)                      \
    S(INIT) F(INIT, deviceId) F(INIT, verbose)                                                        \
    S(CBINFO) F(CBINFO, input_file_name) F(CBINFO, outputFileNameIsRelative) F(CBINFO, output_file_name) \
    F(CBINFO, encoder_parameters) F(CBINFO, image) F(CBINFO, tile) F(CBINFO, error_code)              \
    S(MINPF_REG) F(MINPF_REG, version) F(MINPF_REG, createFunc) F(MINPF_REG, destroyFunc)            \
    S(MINPF_SVC) F(MINPF_SVC, version) F(MINPF_SVC, registerObject) F(MINPF_SVC, invokeService)            \
    S(HINFO) F(HINFO, cblockw_init) F(HINFO, irreversible) F(HINFO, mct) F(HINFO, rsiz) F(HINFO, numresolutions) \
    F(HINFO, csty) F(HINFO, cblk_sty) F(HINFO, prcw_init) F(HINFO, prch_init) F(HINFO, cp_tx0) F(HINFO, cp_th)   \
    F(HINFO, tcp_numlayers) F(HINFO, enumcs) F(HINFO, color) F(HINFO, xml_data) F(HINFO, xml_data_len)        \
    F(HINFO, num_comments) F(HINFO, comment) F(HINFO, comment_len) F(HINFO, isBinaryComment)                  \
    F(HINFO, has_capture_resolution) F(HINFO, capture_resolution) F(HINFO, has_display_resolution)            \
    F(HINFO, display_resolution)                                                                              \
    S(DPARAMS) F(DPARAMS, cp_reduce) F(DPARAMS, cp_layer) F(DPARAMS, infile) F(DPARAMS, outfile)              \
    F(DPARAMS, decod_format) F(DPARAMS, cod_format) F(DPARAMS, DA_x0) F(DPARAMS, DA_y1) F(DPARAMS, m_verbose) \
    F(DPARAMS, tile_index) F(DPARAMS, nb_tile_to_decode) F(DPARAMS, flags)                                    \
    S(DECOMP) F(DECOMP, core) F(DECOMP, infile) F(DECOMP, outfile) F(DECOMP, decod_format) F(DECOMP, cod_format) \
    F(DECOMP, indexfilename) F(DECOMP, DA_x0) F(DECOMP, DA_x1) F(DECOMP, DA_y0) F(DECOMP, DA_y1)              \
    F(DECOMP, m_verbose) F(DECOMP, tile_index) F(DECOMP, nb_tile_to_decode) F(DECOMP, precision)              \
    F(DECOMP, nb_precision) F(DECOMP, force_rgb) F(DECOMP, serialize_xml) F(DECOMP, compression)              \
    F(DECOMP, compressionLevel) F(DECOMP, deviceId) F(DECOMP, repeats) F(DECOMP, verbose) F(DECOMP, numThreads) \
    S(DCBINFO) F(DCBINFO, deviceId) F(DCBINFO, init_decoders_func) F(DCBINFO, inputFile) F(DCBINFO, outputFile) \
    F(DCBINFO, decod_format) F(DCBINFO, cod_format) F(DCBINFO, l_stream) F(DCBINFO, l_codec)                  \
    F(DCBINFO, decoder_parameters) F(DCBINFO, header_info) F(DCBINFO, image) F(DCBINFO, plugin_owns_image)    \
    F(DCBINFO, tile) F(DCBINFO, error_code) F(DCBINFO, decode_flags)                                        \
    S(TCCPINFO) F(TCCPINFO, compno) F(TCCPINFO, csty) F(TCCPINFO, numresolutions) F(TCCPINFO, cblkw)          \
    F(TCCPINFO, cblkh) F(TCCPINFO, cblk_sty) F(TCCPINFO, qmfbid) F(TCCPINFO, qntsty)                         \
    F(TCCPINFO, stepsizes_mant) F(TCCPINFO, stepsizes_expn) F(TCCPINFO, numgbits) F(TCCPINFO, roishift)      \
    F(TCCPINFO, prcw) F(TCCPINFO, prch)                                                                      \
    S(TILEINFO2) F(TILEINFO2, tileno) F(TILEINFO2, csty) F(TILEINFO2, prg) F(TILEINFO2, numlayers)           \
    F(TILEINFO2, mct) F(TILEINFO2, tccp_info)                                                                \
    S(CSINFO) F(CSINFO, tx0) F(CSINFO, ty0) F(CSINFO, tdx) F(CSINFO, tdy) F(CSINFO, tw) F(CSINFO, th)         \
    F(CSINFO, nbcomps) F(CSINFO, m_default_tile_info) F(CSINFO, tile_info)                                   \
    S(MARKER) F(MARKER, type) F(MARKER, pos) F(MARKER, len)                                                  \
    S(TPIDX) F(TPIDX, start_pos) F(TPIDX, end_header) F(TPIDX, end_pos)                                      \
    S(PKTINFO) F(PKTINFO, start_pos) F(PKTINFO, end_ph_pos) F(PKTINFO, end_pos) F(PKTINFO, disto)              \
    S(TILEIDX) F(TILEIDX, tileno) F(TILEIDX, nb_tps) F(TILEIDX, current_nb_tps) F(TILEIDX, current_tpsno)      \
    F(TILEIDX, tp_index) F(TILEIDX, marknum) F(TILEIDX, marker) F(TILEIDX, maxmarknum) F(TILEIDX, nb_packet)   \
    F(TILEIDX, packet_index)                                                                                 \
    S(CSIDX) F(CSIDX, main_head_start) F(CSIDX, main_head_end) F(CSIDX, codestream_size) F(CSIDX, marknum)    \
    F(CSIDX, marker) F(CSIDX, maxmarknum) F(CSIDX, nb_of_tiles) F(CSIDX, tile_index)

#define ABI_EMIT_S(tag) {#tag, "sizeof", sizeof(T_##tag)},
#define ABI_EMIT_F(tag, field) {#tag, #field, offsetof(T_##tag, field)},

struct AbiEntry {
    const char *type, *field;
    size_t value;
};
