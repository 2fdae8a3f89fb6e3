"""ctypes binding of libfsagg.so (the C ABI declared in include/fsagg.h).

The HIP library is the only compute path of this package: importing it on a
machine where the library is missing raises immediately — there is no CPU or
PyTorch fallback anywhere in ``federatedscope_amd``.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get('FSAGG_LIB',
                          os.path.join(_HERE, 'lib', 'libfsagg.so'))

FSAGG_F32, FSAGG_F16, FSAGG_BF16, FSAGG_F64, FSAGG_I64 = range(5)

_c_p = ctypes.c_void_p
_c_i = ctypes.c_int
_c_i64 = ctypes.c_int64
_c_f = ctypes.c_float
_c_sz = ctypes.c_size_t

# name -> (restype, argtypes); mirrors include/fsagg.h one for one
SIGNATURES = {
    'fsagg_version': (_c_i, []),
    'fsagg_last_error': (ctypes.c_char_p, []),
    'fsagg_weighted_sum_f32': (_c_i, [_c_p, _c_p, _c_p, _c_i, _c_i64, _c_p,
                                      _c_p, _c_p]),
    'fsagg_weighted_sum_typed': (_c_i, [_c_p, _c_i, _c_p, _c_i, _c_i64, _c_p,
                                        _c_p]),
    'fsagg_online_inc_f32': (_c_i, [_c_p, _c_p, _c_f, _c_f, _c_f, _c_i64,
                                    _c_p]),
    'fsagg_add_f32': (_c_i, [_c_p, _c_p, _c_p, _c_i64, _c_p]),
    'fsagg_coord_median_f32': (_c_i, [_c_p, _c_i, _c_i64, _c_p, _c_p, _c_p]),
    'fsagg_trimmed_mean_f32': (_c_i, [_c_p, _c_i, _c_i64, _c_i, _c_f, _c_p,
                                      _c_p, _c_p]),
    'fsagg_pairdist_workspace_bytes': (_c_sz, [_c_i, _c_i64, _c_i]),
    'fsagg_pairdist_chunk_elems': (_c_i64, [_c_i, _c_i64, _c_i]),
    'fsagg_pairdist_f32': (_c_i, [_c_p, _c_i, _c_i64, _c_p, _c_i, _c_p, _c_p,
                                  _c_sz, _c_p]),
    'fsagg_pairdist_segsq_f32': (_c_i, [_c_p, _c_i, _c_i64, _c_p, _c_i, _c_p,
                                        _c_p, _c_sz, _c_p]),
    'fsagg_pairdist_finish_f64': (_c_i, [_c_p, _c_i, _c_i, _c_p, _c_p]),
    'fsagg_rownorm_workspace_bytes': (_c_sz, [_c_i, _c_i64]),
    'fsagg_row_sqnorm_f32': (_c_i, [_c_p, _c_i, _c_i64, _c_p, _c_p, _c_sz,
                                    _c_p]),
    'fsagg_fill_uniform_f32': (_c_i, [_c_p, _c_i, _c_i64, _c_i64,
                                      ctypes.c_uint64, _c_i64, _c_p]),
}



_c_d = ctypes.c_double


class OptParams(ctypes.Structure):
    """struct fsagg_opt_params (include/fsagg.h)."""
    _fields_ = [('kind', _c_i), ('flags', _c_i), ('lr', _c_d),
                ('momentum', _c_d), ('dampening', _c_d),
                ('weight_decay', _c_d), ('beta1', _c_d), ('beta2', _c_d),
                ('eps', _c_d), ('step_size', _c_d),
                ('bias_correction2_sqrt', _c_d), ('alpha', _c_d),
                ('clr', _c_d), ('decay_mul', _c_d)]


FSAGG_OPT_SGD, FSAGG_OPT_ADAM, FSAGG_OPT_ADAGRAD, FSAGG_OPT_RMSPROP = range(4)
FSAGG_OPT_NESTEROV, FSAGG_OPT_FIRST_STEP, FSAGG_OPT_AMSGRAD = 1, 2, 4
FSAGG_OPT_DECOUPLED, FSAGG_OPT_MAXIMIZE, FSAGG_OPT_CENTERED = 8, 16, 32
SIGNATURES['fsagg_server_opt_step_f32'] = (
    _c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, ctypes.POINTER(OptParams),
           _c_p])
SIGNATURES['fsagg_server_opt_step_f64'] = (
    _c_i, [_c_p, _c_p, _c_p, _c_p, _c_p, _c_i64, ctypes.POINTER(OptParams),
           _c_p])

FSAGG_WIRE_F32, FSAGG_WIRE_I8, FSAGG_WIRE_I16 = 0, 1, 2
FSAGG_WIRE_B64_F32, FSAGG_WIRE_ZERO = 3, 4
SIGNATURES['fsagg_b64_unpack_f32'] = (
    _c_i, [_c_p, _c_i64, _c_p, _c_i, _c_i64, _c_p, _c_i64, _c_p, _c_p])
SIGNATURES['fsagg_wire_unpack_f32'] = (
    _c_i, [_c_p, _c_i64, _c_p, _c_p, _c_i, _c_i, _c_i64, _c_p, _c_i64, _c_p])
SIGNATURES['fsagg_ss_recover_f32'] = (
    _c_i, [_c_p, _c_p, _c_i, _c_i64, _c_d, _c_d, _c_d, _c_d, _c_d, _c_i, _c_p,
           _c_p, _c_p])
SIGNATURES['fsagg_delta_sqnorm_workspace_bytes'] = (_c_sz, [_c_i, _c_i64,
                                                            _c_i])
SIGNATURES['fsagg_delta_wsum_f32'] = (
    _c_i, [_c_p, _c_p, _c_i, _c_i64, _c_p, _c_p, _c_p])
SIGNATURES['fsagg_delta_sqnorm_f32'] = (
    _c_i, [_c_p, _c_i, _c_i64, _c_p, _c_p, _c_i, _c_p, _c_p, _c_sz, _c_p])
SIGNATURES['fsagg_delta_sqnorm_keys_f32'] = (
    _c_i, [_c_p, _c_i, _c_i64, _c_p, _c_p, _c_i, _c_p, _c_p, _c_sz, _c_p])
SIGNATURES['fsagg_delta_wsum_keys_f32'] = (
    _c_i, [_c_p, _c_p, _c_i, _c_i64, _c_p, _c_p, _c_i, _c_p, _c_p])
SIGNATURES['fsagg_delta_sqnorm_wsum_workspace_bytes'] = (
    _c_sz, [_c_i, _c_i64, _c_i])
SIGNATURES['fsagg_delta_sqnorm_wsum_f32'] = (
    _c_i, [_c_p, _c_p, _c_i, _c_i64, _c_p, _c_p, _c_i, _c_p, _c_p, _c_p,
           _c_sz, _c_p])
SIGNATURES['fsagg_delta_sqnorm_wsum_keys_f32'] = (
    _c_i, [_c_p, _c_p, _c_i, _c_i64, _c_p, _c_p, _c_i, _c_p, _c_p, _c_p,
           _c_sz, _c_p])
FSAGG_STACK_CHUNK = 2048
SIGNATURES['fsagg_gather_rows_f32'] = (
    _c_i, [_c_p, _c_i, _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_i, _c_p])



class Rows(ctypes.Structure):
    """struct fsagg_rows (include/fsagg.h): a row set's pointer table."""
    _fields_ = [('tab', _c_p), ('ss', _c_i64), ('n', _c_i), ('nseg', _c_i)]


_rows_p = ctypes.POINTER(Rows)
FSAGG_ROWS_OS_CHUNK = 256
SIGNATURES['fsagg_wsum_chunk_elems'] = (_c_i64, [_c_i64])
SIGNATURES['fsagg_wsum_chunk_elems_n'] = (_c_i64, [_c_i64, _c_i])
SIGNATURES['fsagg_wsum_set_rows_width'] = (_c_i, [_c_i])
SIGNATURES['fsagg_weighted_sum_rows_f32'] = (
    _c_i, [_rows_p, _c_p, _c_i, _c_i64, _c_p, _c_p, _c_p, _c_i64, _c_p, _c_p])
SIGNATURES['fsagg_coord_median_rows_f32'] = (
    _c_i, [_rows_p, _c_p, _c_i, _c_i64, _c_p, _c_i64, _c_p, _c_p])
SIGNATURES['fsagg_orderstat_set_pair_min'] = (_c_i, [_c_i])
SIGNATURES['fsagg_orderstat_set_group_max'] = (_c_i, [_c_i])
SIGNATURES['fsagg_orderstat_set_group_range'] = (_c_i, [_c_i, _c_i])
SIGNATURES['fsagg_orderstat_set_group_waves'] = (_c_i, [_c_i])
SIGNATURES['fsagg_trimmed_mean_rows_f32'] = (
    _c_i, [_rows_p, _c_p, _c_i, _c_i64, _c_i, _c_f, _c_p, _c_i64, _c_p,
           _c_p])
SIGNATURES['fsagg_pairgram_workspace_bytes'] = (_c_sz, [_c_i, _c_i64, _c_i])
SIGNATURES['fsagg_pairgram_set_block8'] = (_c_i, [_c_i])
SIGNATURES['fsagg_pairgram_block8'] = (_c_i, [])
SIGNATURES['fsagg_pairgram_set_stages'] = (_c_i, [_c_i])
SIGNATURES['fsagg_pairgram_set_chunks'] = (_c_i, [_c_i])
SIGNATURES['fsagg_pairgram_set_desync'] = (_c_i, [_c_i])
SIGNATURES['fsagg_pairgram_set_fused'] = (_c_i, [_c_i])
SIGNATURES['fsagg_pairgram_knobs'] = (_c_i64, [])
SIGNATURES['fsagg_pairgram_rows_segsq_f32'] = (
    _c_i, [_c_p, _c_p, _c_p, _c_i64, _c_p, _c_p, _c_p, _c_sz, _c_p])
SIGNATURES['fsagg_pairgram_rows_f32'] = (
    _c_i, [_c_p, _c_p, _c_p, _c_i64, ctypes.c_double, _c_p, _c_p, _c_p, _c_p,
           _c_p, _c_p, _c_p, _c_sz, _c_p])
SIGNATURES['fsagg_pairgram_finish_f32'] = (
    _c_i, [_c_p, _c_p, _c_i, _c_i, ctypes.c_double, _c_p, _c_p, _c_p, _c_p,
           _c_p])
SIGNATURES['fsagg_pairdist_rows_segsq_f32'] = (
    _c_i, [_rows_p, _c_p, _c_p, _c_i64, _c_p, _c_p, _c_sz, _c_p])
SIGNATURES['fsagg_pairsel_workspace_bytes'] = (_c_sz, [_c_i, _c_i, _c_i])
SIGNATURES['fsagg_pairsel_rows_segsq_f64'] = (
    _c_i, [_rows_p, _c_p, _c_i, _c_p, _c_i, _c_p, _c_p, _c_sz, _c_p])
SIGNATURES['fsagg_pairsel_finish_f64'] = (
    _c_i, [_c_p, _c_p, _c_i, _c_i, _c_i, _c_p, _c_p])
FSAGG_PAIRSEL_MAX_SEL = 32
FSAGG_PAIRSEL_MAX_CLIENTS = 256
FSAGG_PAIRSEL_CHUNK = 2048

SIGNATURES['fsagg_online_inc_typed'] = (
    _c_i, [_c_p, _c_i, _c_p, _c_i, _c_p, _c_i, _c_i64, _c_i64, _c_i64, _c_p])
SIGNATURES['fsagg_rows_sqnorm_workspace_bytes'] = (_c_sz, [_c_i, _c_i])
SIGNATURES['fsagg_rows_sqnorm_f32'] = (
    _c_i, [_rows_p, _c_p, _c_i, _c_p, _c_p, _c_sz, _c_p])
SIGNATURES['fsagg_normbound_prescale_f32'] = (
    _c_i, [_c_p, _c_i, _c_i, ctypes.c_float, _c_p, _c_p])

FSAGG_MAX_PEERS = 8
FSAGG_PAIRGRAM_MAX_CLIENTS = 256
_c_u32 = ctypes.c_uint32
SIGNATURES['fsagg_peer_handle_bytes'] = (_c_sz, [])
SIGNATURES['fsagg_peer_alloc'] = (_c_i, [_c_i, _c_sz, ctypes.POINTER(_c_p)])
SIGNATURES['fsagg_peer_free'] = (_c_i, [_c_i, _c_p])
SIGNATURES['fsagg_peer_status_alloc'] = (
    _c_i, [ctypes.POINTER(_c_p), ctypes.POINTER(_c_p)])
SIGNATURES['fsagg_peer_status_free'] = (_c_i, [_c_p])
SIGNATURES['fsagg_peer_handle'] = (_c_i, [_c_p, _c_p])
SIGNATURES['fsagg_peer_open'] = (_c_i, [_c_i, _c_p, ctypes.POINTER(_c_p)])
SIGNATURES['fsagg_peer_close'] = (_c_i, [_c_i, _c_p])
SIGNATURES['fsagg_peer_pci_bus_id'] = (_c_i, [_c_i, ctypes.c_char_p, _c_i])
SIGNATURES['fsagg_peer_can_access'] = (_c_i, [_c_i, ctypes.c_char_p])
SIGNATURES['fsagg_weighted_sum_bcast_f32'] = (
    _c_i, [_c_p, _c_p, _c_p, _c_i, _c_i64, _c_p, ctypes.POINTER(_c_p), _c_i,
           _c_p])
FSAGG_HOSTTAB_MAX_CLIENTS = 128
FSAGG_HOSTTAB_ROWS_MAX_CLIENTS = 64
FSAGG_KRUMSEL_MAX_CLIENTS = 256
FSAGG_KRUMSEL_MAX_SEGS = 64
SIGNATURES['fsagg_krum_select_f32'] = (
    _c_i, [_c_p, _c_i, _c_i, _c_i, _c_i, _c_i, _c_p, _c_i, _c_p, _c_p, _c_i64,
           _c_i, _c_p, _c_p, _c_p, _c_p, _c_p, _c_p])
FSAGG_HOSTTAB_ROWS_MAX_PTRS = 256
FSAGG_HOSTTAB_ROWS_MAX_SEGS = 64
SIGNATURES['fsagg_weighted_sum_rows_hosttab_f32'] = (
    _c_i, [_c_p, _c_i, _c_i, _c_p, _c_i, _c_i64, _c_p, _c_p, _c_p, _c_p,
           _c_p])
SIGNATURES['fsagg_upload_h2d'] = (
    _c_i, [_c_p, _c_p, _c_sz, _c_p, _c_i, _c_i, _c_p, _c_p])
SIGNATURES['fsagg_upload_wait'] = (_c_i, [_c_i, _c_p])
SIGNATURES['fsagg_fetch_mapped_u64'] = (_c_i, [_c_p, _c_p, _c_i64, _c_p])
SIGNATURES['fsagg_weighted_sum_hosttab_f32'] = (
    _c_i, [_c_p, _c_p, _c_p, _c_i, _c_i64, _c_p, ctypes.POINTER(_c_p), _c_i,
           _c_p])
SIGNATURES['fsagg_peer_push_f32'] = (
    _c_i, [_c_p, ctypes.POINTER(_c_p), _c_i, _c_i64, _c_p])
SIGNATURES['fsagg_peer_barrier'] = (
    _c_i, [ctypes.POINTER(_c_p), _c_i, _c_i, _c_u32, ctypes.c_uint64, _c_p,
           _c_p])

_lib = None
_host = None
HOST_PATH = os.path.join(_HERE, 'lib', '_fsagg_host.so')


def host():
    """The _fsagg_host extension (csrc/host/keytable.cpp): builds row-set
    pointer tables from client state_dicts in C++.  Raises FsaggError if it
    was not built."""
    global _host
    if _host is None:
        if not os.path.exists(HOST_PATH):
            raise FsaggError('_fsagg_host.so not found at %s — build with '
                             'make -C federatedscope_amd/csrc' % HOST_PATH)
        import importlib.util
        import torch  # noqa: F401  (libtorch_python first)
        spec = importlib.util.spec_from_file_location('_fsagg_host',
                                                      HOST_PATH)
        mod = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(mod)
        _host = mod
    return _host


class FsaggError(RuntimeError):
    pass


def load(path=None):
    """Load libfsagg.so (once).  Raises FsaggError if it is missing."""
    global _lib
    if _lib is not None:
        return _lib
    p = path or LIB_PATH
    if not os.path.exists(p):
        raise FsaggError(
            'libfsagg.so not found at %s — build it with '
            '`python -c "import __graft_entry__ as g; g.build()"` '
            '(make -C federatedscope_amd/csrc).  federatedscope_amd has no '
            'CPU fallback.' % p)
    # torch first: its bundled libamdhip64.so.7 then satisfies our NEEDED
    # entry, so the library and torch share one HIP runtime (one set of
    # streams / device pointers).
    import torch  # noqa: F401
    lib = ctypes.CDLL(p, mode=ctypes.RTLD_GLOBAL)
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    _lib = lib
    return lib


def check(rc, what=''):
    if rc != 0:
        msg = load().fsagg_last_error()
        raise FsaggError('%s failed (%d): %s' %
                         (what, rc, msg.decode() if msg else ''))
    return rc


def exported_symbols():
    return list(SIGNATURES.keys())
