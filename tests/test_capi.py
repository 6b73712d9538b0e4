

def test_coord_raw_option_is_per_thread():
    """coord_raw (raw-coordinate shooting kernels) is a per-host-thread library option: the
    shooting sets it around its own launches, concurrent frames run on their own threads."""
    import threading
    from difficp_amd import _lib
    assert _lib.get_option("coord_raw") == 0
    seen = []
    with _lib.coord_mode(True):
        assert _lib.get_option("coord_raw") == 1
        t = threading.Thread(target=lambda: seen.append(_lib.get_option("coord_raw")))
        t.start()
        t.join()
    assert seen == [0] and _lib.get_option("coord_raw") == 0
