// Material.h — host-side material description with the reference API
// (Core/Material.cuh:8-47: MaterialType, MaterialData).  The device-side
// virtual Material classes of the reference (:49-150) are replaced by a tagged
// material table evaluated inside the render kernel.
#pragma once
#include "Vec3.h"

namespace CRT {

enum class MaterialType : int { Lambertian = 0, Metal = 1, Dielectric = 2, DiffuseLight = 3 };

class MaterialData {
public:
    MaterialData() : m_Type(MaterialType::Lambertian), m_Albedo(0.f), m_Emission(0.f), m_Roughness(0.f), m_IOR(1.f) {}
    MaterialData(MaterialType type, const Vec3& albedo, float roughness, float ior, const Vec3& emission)
        : m_Type(type), m_Albedo(albedo), m_Emission(emission), m_Roughness(roughness), m_IOR(ior) {}
    MaterialType getType() const { return m_Type; }
    Vec3 getAlbedo() const { return m_Albedo; }
    Vec3 getEmission() const { return m_Emission; }
    float getRoughness() const { return m_Roughness; }
    float getIOR() const { return m_IOR; }

private:
    MaterialType m_Type;
    Vec3 m_Albedo;
    Vec3 m_Emission;
    float m_Roughness;
    float m_IOR;
};

}  // namespace CRT
