-- Shape from shading: refine a depth map X so that its spherical-harmonics shading
-- matches an intensity image (same energy as the reference's
-- examples/shape_from_shading/shape_from_shading.t; declaration indices identical).
local W, H = Dim("W", 0), Dim("H", 1)

local sqrt_wp = sqrt(Param("w_p", float, 0))   -- depth fit
local sqrt_ws = sqrt(Param("w_s", float, 1))   -- smoothness
local sqrt_wg = sqrt(Param("w_g", float, 2))   -- shading
local fx, fy = Param("f_x", float, 3), Param("f_y", float, 4)
local cx, cy = Param("u_x", float, 5), Param("u_y", float, 6)
local sh = {}
for k = 1, 9 do sh[k] = Param("L_" .. k, float, 6 + k) end  -- lighting coefficients

local Z = Unknown("X", opt_float, {W, H}, 16)            -- refined depth
local Z_in = Array("D_i", opt_float, {W, H}, 17)          -- input depth (<= 0: no data)
local intensity = Array("Im", opt_float, {W, H}, 18)
local edge_row = Array("edgeMaskR", uint8, {W, H}, 19)
local edge_col = Array("edgeMaskC", uint8, {W, H}, 20)

local x, y = Index(0), Index(1)

local function has_depth(dx, dy) return greater(Z_in(dx, dy), 0) end

-- back-projected point of pixel (x+dx, y+dy)
local function point(dx, dy)
    local z = Z(dx, dy)
    return Vector(((dx + x - cx) / fx) * z, ((dy + y - cy) / fy) * z, z)
end

-- unit normal from the left / upper neighbours
local function normal(dx, dy)
    local zc, zl, zu = Z(dx, dy), Z(dx - 1, dy), Z(dx, dy - 1)
    local nx = zu * (zc - zl) / fy
    local ny = zl * (zc - zu) / fx
    local nz = (nx * (cx - (x + dx)) / fx) + (ny * (cy - (y + dy)) / fy) - (zl * zu / (fx * fy))
    local len2 = nx * nx + ny * ny + nz * nz
    local s = Select(greater(len2, 0.0), 1.0 / sqrt(len2), 1.0)
    return s * Vector(nx, ny, nz)
end

local function shading(dx, dy)
    local n = normal(dx, dy)
    local a, b, c = n[0], n[1], n[2]
    return sh[1] + sh[2] * b + sh[3] * c + sh[4] * a + sh[5] * a * b + sh[6] * b * c
         + sh[7] * (-a * a - b * b + 2 * c * c) + sh[8] * c * a + sh[9] * (a * a - b * b)
end

local function target(dx, dy)
    return intensity(dx, dy) * 0.5 + 0.25 * (intensity(dx - 1, dy) + intensity(dx, dy - 1))
end

local shading_error = ComputedArray("B_I", {W, H},
    Select(InBoundsExpanded(0, 0, 1) * (has_depth(-1, 0) * has_depth(0, 0) * has_depth(0, -1)),
           shading(0, 0) - target(0, 0), 0))

Exclude(Not(has_depth(0, 0)))

Energy(Select(has_depth(0, 0), sqrt_wp * (Z(0, 0) - Z_in(0, 0)), 0))

Energy(Select(InBoundsExpanded(0, 0, 1),
              sqrt_wg * ((shading_error(0, 0) - shading_error(1, 0)) * edge_row(0, 0)), 0))
Energy(Select(InBoundsExpanded(0, 0, 1),
              sqrt_wg * ((shading_error(0, 0) - shading_error(0, 1)) * edge_col(0, 0)), 0))

local function smooth_to(dx, dy) return less(abs(Z(0, 0) - Z(dx, dy)), 0.01) end
local smooth_ok = ComputedArray("valid", {W, H},
    has_depth(0, 0) * has_depth(0, -1) * has_depth(0, 1) * has_depth(-1, 0) * has_depth(1, 0) *
    smooth_to(0, -1) * smooth_to(0, 1) * smooth_to(-1, 0) * smooth_to(1, 0) * InBoundsExpanded(0, 0, 1))
local laplacian = 4.0 * point(0, 0) - (point(-1, 0) + point(0, -1) + point(1, 0) + point(0, 1))
Energy(Select(eq(smooth_ok(0, 0), 1), sqrt_ws * laplacian, 0))
