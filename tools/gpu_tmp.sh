timeout -k 10 200 python tools/layer_profile.py
