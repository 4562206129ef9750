class Array:
  def __init__(self, *a, **k):
    pass


class BoundedArray(Array):
  pass
