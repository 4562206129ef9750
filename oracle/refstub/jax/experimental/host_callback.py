def call(f, arg, **_):
  return f(arg)
