// tv_options_internal.h -- option keys of libtorrent_verify.so that are NOT part of its public ABI
// (include/torrent_verify.h): measurement and test knobs (A/B builds, probes, fault injection).  The tests and the
// tools set them through tv_set_option with these values; a host integrating the library never needs them.
#pragma once
