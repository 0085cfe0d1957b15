python tools/single_loop.py c4 200
python tools/single_loop.py c4i 200
python tools/single_loop.py c4 200
python tools/single_loop.py c4i 200
python tools/walk_stamps.py mixed
python tools/walk_stamps.py 1k
