def init_from_env():
    return None
