"""python -m torrent_amd verify <file.torrent> <dir> [--devices N]
Resume check from disk: prints the have-bitfield summary of the files under <dir> (verify_files)."""
import sys


def main(argv=None) -> int:
    args = list(sys.argv[1:] if argv is None else argv)
    if len(args) < 3 or args[0] != "verify":
        print(__doc__)
        return 2
    from .metainfo import parse_metainfo
    from .verify import verify_files
    devices = 1
    if "--devices" in args:
        devices = int(args[args.index("--devices") + 1])
    meta = parse_metainfo(open(args[1], "rb").read())
    if meta is None:
        print("invalid .torrent file")
        return 1
    bf = verify_files(meta.info, args[2], devices=devices)
    P = meta.info.n_pieces
    have = sum(bin(b).count("1") for b in bf)
    print(f"{have}/{P} pieces verified")
    print(bytes(bf).hex())
    return 0 if have == P else 1


if __name__ == "__main__":
    raise SystemExit(main())
